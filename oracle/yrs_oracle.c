/*
 * yrs_oracle.c — TEST INFRASTRUCTURE ONLY (see yrs_oracle.h).
 *
 * A plain-C restatement of yrs 0.19.2's binary-update algebra over lib0 v1:
 *   merge_updates_v1                    yrs/src/alt.rs:15-28,  yrs/src/update.rs:537-704
 *   diff_updates_v1                     yrs/src/alt.rs:73-81,  yrs/src/update.rs:490-535
 *   encode_state_vector_from_update_v1  yrs/src/alt.rs:54-57,  yrs/src/update.rs:107-114
 * with the lib0 primitives (yrs/src/encoding/varint.rs:184-281, read.rs:84-172),
 * the v1 block/content codec (yrs/src/update.rs:433-488, yrs/src/block.rs:1711-1835,
 * yrs/src/slice.rs:199-251, yrs/src/any.rs:37-183), DeleteSet/IdRange
 * (yrs/src/id_set.rs:18-426) and an emulation of std's hashbrown SwissTable
 * iteration order under ClientHasher (yrs/src/utils/client_hasher.rs) which fixes
 * the order DeleteSet and StateVector clients are written in.
 *
 * Policies where yrs is not deterministic or not total (documented in DESIGN.md):
 *  - Any::Map is a RandomState HashMap in yrs (any.rs:23): a repeated key keeps its last
 *    value and each distinct key is written at its last occurrence.  Doc options
 *    (doc.rs:814) are rebuilt in as_any order.
 *  - allocation failures: a fallible try_reserve fails (NotEnoughMemory) and an
 *    infallible with_capacity aborts (REFERENCE_PANIC) when it would need more
 *    than 2^36 bytes.
 *  - Item-vs-GC ties at one (client, clock) make yrs' comparator inconsistent
 *    (update.rs:580-582).  With <= 20 live decoders Rust's stable sort_by IS
 *    insertion_sort_shift_left in every std version, and we follow it literally
 *    (pinned).  Above 20 the outcome depends on the std version's sort algorithm
 *    (merge sort before Rust 1.81, driftsort after, which may even panic): unpinned,
 *    and our policy is the stable sort under the consistent comparator that treats
 *    the Item/GC tie as Equal (update.rs:580's same_type arm) — see merge_blocks.
 *  - Embed/Format JSON goes through the serde_json + ryu restatement below (JSON section);
 *    objects with >= 2 distinct keys are RandomState-ordered in yrs: written at each key's
 *    last occurrence (the same policy as Any maps above).
 */
#include "yrs_oracle.h"

#include <math.h>
#include <stdio.h>
#include <pthread.h>
#include <stdbool.h>
#include <stdlib.h>
#include <string.h>

#define ALLOC_LIMIT (1ull << 36)
#define TRY(x)                                                                                     \
  do {                                                                                             \
    int _e = (x);                                                                                  \
    if (_e) return _e;                                                                             \
  } while (0)

/* ------------------------------------------------------------------ vectors */
#define VEC(T)                                                                                     \
  struct {                                                                                         \
    T *d;                                                                                          \
    size_t n, cap;                                                                                 \
  }
#define VGROW(v, need)                                                                             \
  do {                                                                                             \
    if ((need) > (v).cap) {                                                                        \
      size_t _c = (v).cap ? (v).cap : 8;                                                           \
      while (_c < (need)) _c *= 2;                                                                 \
      (v).d = realloc((v).d, _c * sizeof(*(v).d));                                                 \
      (v).cap = _c;                                                                                \
    }                                                                                              \
  } while (0)
#define VPUSH(v, x)                                                                                \
  do {                                                                                             \
    VGROW(v, (v).n + 1);                                                                           \
    (v).d[(v).n++] = (x);                                                                          \
  } while (0)
#define VFREE(v)                                                                                   \
  do {                                                                                             \
    free((v).d);                                                                                   \
    (v).d = NULL;                                                                                  \
    (v).n = (v).cap = 0;                                                                           \
  } while (0)

/* ------------------------------------------------------------------ reader (read.rs:36-82) */
typedef struct {
  const uint8_t *p;
  size_t n, i;
} rd_t;

static int rd_u8(rd_t *r, uint8_t *v) {
  if (r->i >= r->n) return YO_ERR_EOS;
  *v = r->p[r->i++];
  return 0;
}
static int rd_exact(rd_t *r, uint64_t len, const uint8_t **s) {
  if (len > r->n - r->i) return YO_ERR_EOS;
  *s = r->p + r->i;
  r->i += (size_t)len;
  return 0;
}
/* varint.rs:244-260: u32 with wrapping_shl, up to 11 bytes */
static int rd_var_u32(rd_t *r, uint32_t *v) {
  uint32_t num = 0;
  unsigned len = 0;
  for (;;) {
    uint8_t b;
    TRY(rd_u8(r, &b));
    num |= (uint32_t)(b & 0x7f) << (len & 31);
    len += 7;
    if (b < 0x80) {
      *v = num;
      return 0;
    }
    if (len > 70) return YO_ERR_VAR_INT;
  }
}
/* varint.rs:228-242 */
static int rd_var_u64(rd_t *r, uint64_t *v) {
  uint64_t num = 0;
  unsigned len = 0;
  for (;;) {
    uint8_t b;
    TRY(rd_u8(r, &b));
    num |= (uint64_t)(b & 0x7f) << (len & 63);
    len += 7;
    if (b < 0x80) {
      *v = num;
      return 0;
    }
    if (len > 70) return YO_ERR_VAR_INT;
  }
}
/* varint.rs:262-281: lib0 signed varint, sign in bit 6 of the first byte */
static int rd_var_i64(rd_t *r, int64_t *v) {
  uint8_t b;
  TRY(rd_u8(r, &b));
  uint64_t num = b & 0x3f;
  unsigned len = 6;
  bool neg = (b & 0x40) != 0;
  if (!(b & 0x80)) {
    *v = neg ? (int64_t)(0 - num) : (int64_t)num;
    return 0;
  }
  for (;;) {
    TRY(rd_u8(r, &b));
    num |= (uint64_t)(b & 0x7f) << (len & 63);
    len += 7;
    if (b < 0x80) {
      *v = neg ? (int64_t)(0 - num) : (int64_t)num;
      return 0;
    }
    if (len > 70) return YO_ERR_VAR_INT;
  }
}
/* read_buf / read_string (read.rs:100-104,131-135): u32 length prefix */
static int rd_buf(rd_t *r, const uint8_t **s, uint32_t *len) {
  TRY(rd_var_u32(r, len));
  return rd_exact(r, *len, s);
}

/* ------------------------------------------------------------------ writer (write.rs, varint.rs:184-226) */
typedef struct {
  uint8_t *d;
  size_t n, cap;
} wb_t;
static void wb_u8(wb_t *w, uint8_t b) {
  VGROW(*w, w->n + 1);
  w->d[w->n++] = b;
}
static void wb_bytes(wb_t *w, const uint8_t *s, size_t n) {
  VGROW(*w, w->n + n);
  if (n) memcpy(w->d + w->n, s, n);
  w->n += n;
}
static void wb_var(wb_t *w, uint64_t v) {
  while (v >= 0x80) {
    wb_u8(w, (uint8_t)((v & 0x7f) | 0x80));
    v >>= 7;
  }
  wb_u8(w, (uint8_t)v);
}
static void wb_var_i64(wb_t *w, int64_t value) {
  bool neg = value < 0;
  if (neg) value = (int64_t)(0 - (uint64_t)value);
  wb_u8(w, (uint8_t)((value > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (uint8_t)(63 & value)));
  value >>= 6;
  while (value > 0) {
    wb_u8(w, (uint8_t)((value > 127 ? 0x80 : 0) | (uint8_t)(127 & value)));
    value >>= 7;
  }
}
static void wb_str(wb_t *w, const uint8_t *s, uint32_t n) {
  wb_var(w, n);
  wb_bytes(w, s, n);
}

/* ------------------------------------------------------------------ hashbrown emulation
 * std HashMap<u64, _, BuildHasherDefault<ClientHasher>>: hash = key, h1 = hash & mask,
 * SSE2 group width 16, iteration = ascending bucket index.  Only insertions happen. */
typedef struct {
  size_t buckets; /* 0 = unallocated empty singleton */
  size_t items, growth_left;
  int32_t *slot; /* bucket -> entry index, -1 empty */
  VEC(uint64_t) keys;
} hb_t;

static size_t cap_to_buckets(size_t cap) {
  if (cap < 8) return cap < 4 ? 4 : 8;
  size_t adj = cap * 8 / 7, b = 1;
  while (b < adj) b <<= 1;
  return b;
}
static size_t mask_to_cap(size_t mask) { return mask < 8 ? mask : ((mask + 1) / 8) * 7; }
static bool hb_ctrl_empty(const hb_t *t, size_t idx) {
  if (idx < t->buckets) return t->slot[idx] < 0;
  if (t->buckets < 16) return idx < 16 ? true : t->slot[idx - 16] < 0;
  return t->slot[idx - t->buckets] < 0;
}
static size_t hb_find_insert_slot(const hb_t *t, uint64_t hash) {
  size_t mask = t->buckets - 1, pos = (size_t)hash & mask, stride = 0;
  for (;;) {
    for (size_t j = 0; j < 16; j++) {
      if (hb_ctrl_empty(t, pos + j)) {
        size_t index = (pos + j) & mask;
        if (t->slot[index] >= 0) { /* fix_insert_slot: small-table trailing EMPTY */
          for (size_t k = 0; k < t->buckets; k++)
            if (t->slot[k] < 0) return k;
        }
        return index;
      }
    }
    stride += 16;
    pos = (pos + stride) & mask;
  }
}
static int32_t hb_find(const hb_t *t, uint64_t key) {
  if (!t->buckets) return -1;
  size_t mask = t->buckets - 1, pos = (size_t)key & mask, stride = 0;
  for (;;) {
    bool any_empty = false;
    for (size_t j = 0; j < 16; j++) {
      size_t idx = pos + j;
      if (hb_ctrl_empty(t, idx)) {
        any_empty = true;
        continue;
      }
      int32_t e = t->slot[idx & mask];
      if (e >= 0 && t->keys.d[e] == key) return e;
    }
    if (any_empty) return -1;
    stride += 16;
    pos = (pos + stride) & mask;
  }
}
static void hb_resize(hb_t *t, size_t cap) {
  size_t nb = cap_to_buckets(cap);
  int32_t *ns = malloc(nb * sizeof(int32_t));
  for (size_t i = 0; i < nb; i++) ns[i] = -1;
  hb_t tmp = *t;
  tmp.buckets = nb;
  tmp.slot = ns;
  for (size_t i = 0; i < t->buckets; i++) {
    int32_t e = t->slot[i];
    if (e < 0) continue;
    size_t s = hb_find_insert_slot(&tmp, t->keys.d[e]);
    ns[s] = e;
  }
  free(t->slot);
  t->slot = ns;
  t->buckets = nb;
  t->growth_left = mask_to_cap(nb - 1) - t->items;
}
/* RawTable::reserve / try_reserve; elem = sizeof((K,V)) for the allocation policy */
static int hb_reserve(hb_t *t, uint64_t add, size_t elem, bool fallible) {
  if (add <= t->growth_left) return 0;
  size_t full_cap = t->buckets ? mask_to_cap(t->buckets - 1) : 0;
  uint64_t need = t->items + add;
  uint64_t cap = need > full_cap + 1 ? need : full_cap + 1;
  uint64_t nb = cap < (1ull << 40) ? cap_to_buckets((size_t)cap) : (1ull << 62);
  if (nb * (elem + 1) > ALLOC_LIMIT) return fallible ? YO_ERR_NOT_ENOUGH_MEMORY : YO_ERR_REFERENCE_PANIC;
  hb_resize(t, (size_t)cap);
  return 0;
}
static void hb_place(hb_t *t, uint64_t key, int32_t e) {
  size_t s = hb_find_insert_slot(t, key);
  t->slot[s] = e;
  t->items++;
  t->growth_left--;
}
/* HashMap::insert: reserve(1) first (hashbrown find_or_find_insert_slot), replace if present */
static int32_t hb_insert(hb_t *t, uint64_t key, bool *existed) {
  hb_reserve(t, 1, 0, true);
  int32_t e = hb_find(t, key);
  if (e >= 0) {
    *existed = true;
    return e;
  }
  *existed = false;
  e = (int32_t)t->keys.n;
  VPUSH(t->keys, key);
  hb_place(t, key, e);
  return e;
}
/* HashMap::entry(..).or_insert: reserve(1) only when vacant (rustc_entry) */
static int32_t hb_entry(hb_t *t, uint64_t key, bool *existed) {
  int32_t e = hb_find(t, key);
  if (e >= 0) {
    *existed = true;
    return e;
  }
  *existed = false;
  hb_reserve(t, 1, 0, true);
  e = (int32_t)t->keys.n;
  VPUSH(t->keys, key);
  hb_place(t, key, e);
  return e;
}
static void hb_with_capacity(hb_t *t, size_t n) {
  memset(t, 0, sizeof(*t));
  if (n == 0) return;
  t->buckets = cap_to_buckets(n);
  t->slot = malloc(t->buckets * sizeof(int32_t));
  for (size_t i = 0; i < t->buckets; i++) t->slot[i] = -1;
  t->growth_left = mask_to_cap(t->buckets - 1);
}
/* entry indices in iteration (ascending bucket) order */
static size_t hb_order(const hb_t *t, int32_t *out) {
  size_t k = 0;
  for (size_t i = 0; i < t->buckets; i++)
    if (t->slot[i] >= 0) out[k++] = t->slot[i];
  return k;
}
static void hb_free(hb_t *t) {
  free(t->slot);
  VFREE(t->keys);
  memset(t, 0, sizeof(*t));
}

/* ------------------------------------------------------------------ UTF-8 (core::str next_code_point) */
static uint32_t utf8_next(const uint8_t *s, size_t n, size_t *i) {
#define NB() (*i < n ? s[(*i)++] : (uint8_t)0)
  uint8_t x = s[(*i)++];
  if (x < 128) return x;
  uint32_t init = x & (0x7F >> 2);
  uint8_t y = NB();
  uint32_t ch = (init << 6) | (y & 0x3F);
  if (x >= 0xE0) {
    uint8_t z = NB();
    uint32_t y_z = ((uint32_t)(y & 0x3F) << 6) | (z & 0x3F);
    ch = init << 12 | y_z;
    if (x >= 0xF0) {
      uint8_t w = NB();
      ch = (init & 7) << 18 | ((y_z << 6) | (w & 0x3F));
    }
  }
  return ch;
#undef NB
}
static uint32_t ch_len16(uint32_t c) { return (c & 0xFFFF) == c ? 1 : 2; }
static uint32_t ch_len8(uint32_t c) { return c < 0x80 ? 1 : c < 0x800 ? 2 : c < 0x10000 ? 3 : 4; }
/* SplittableString::len(Utf16) (block.rs:1391-1401) */
static uint32_t str_len16(const uint8_t *s, uint32_t n) {
  if (n == 1) return 1;
  uint32_t k = 0;
  size_t i = 0;
  while (i < n) k += ch_len16(utf8_next(s, n, &i));
  return k;
}
/* split_str(.., Utf16) byte offset (block.rs:1483-1502); str::split_at panics off a
 * char boundary */
static int str_split16(const uint8_t *s, uint32_t n, uint32_t offset, uint32_t *byte_off) {
  uint32_t off = 0, u = 0;
  size_t i = 0;
  while (i < n) {
    if (u >= offset) break;
    uint32_t c = utf8_next(s, n, &i);
    off += ch_len8(c);
    u += ch_len16(c);
  }
  if (off > n || (off < n && (int8_t)s[off] < -0x40)) return YO_ERR_REFERENCE_PANIC;
  *byte_off = off;
  return 0;
}

/* ------------------------------------------------------------------ decoded model */
enum { BK_ITEM = 0, BK_GC = 1, BK_SKIP = 2 };
enum { PK_UNKNOWN = 0, PK_NAMED = 1, PK_ID = 2 };
typedef struct {
  const uint8_t *p;
  uint32_t n;
} span_t;
typedef struct {
  uint8_t kind, ref, has_origin, has_ro, pkind, has_psub, tref, unsupported;
  uint8_t json_any; /* lib0 v2: Embed/Format values are Any bytes (read_json = Any::decode) */
  uint64_t client, oc, rc, pc, sc, ec;
  uint32_t clock, len, ok, rk, pk, sk, ek;
  span_t pname, psub, cs, cs2;
  uint32_t n;  /* Deleted count / element count */
  uint32_t e0; /* first element span (Any / JSON) */
  int64_t mflags;
  /* Doc options */
  uint8_t doc_skip_gc, doc_auto_load, doc_has_cid, doc_enc_bytes;
  span_t doc_cid;
} blk_t;
typedef struct {
  uint32_t s, e;
} rng_t;
typedef struct {
  int cont;
  rng_t c;
  VEC(rng_t) v;
} idr_t;
typedef struct {
  VEC(uint32_t) idx;
} blist_t;
typedef VEC(idr_t) idrvec_t;
typedef struct {
  const uint8_t *base;
  size_t len;
  VEC(blk_t) blocks;
  VEC(span_t) elems;
  hb_t clients; /* UpdateBlocks.clients */
  VEC(blist_t) lists;
  hb_t ds; /* DeleteSet */
  VEC(idr_t) dsv;
  int unsupported;
} upd_t;

static void idr_free(idr_t *r) { VFREE(r->v); }
static void upd_free(upd_t *u) {
  VFREE(u->blocks);
  VFREE(u->elems);
  hb_free(&u->clients);
  for (size_t i = 0; i < u->lists.n; i++) VFREE(u->lists.d[i].idx);
  VFREE(u->lists);
  hb_free(&u->ds);
  for (size_t i = 0; i < u->dsv.n; i++) idr_free(&u->dsv.d[i]);
  VFREE(u->dsv);
}

/* ------------------------------------------------------------------ Any (any.rs:37-83) */
/* Validates one Any value.  Policy shared with the device: a container nested
 * 64 deep -> UNSUPPORTED.  (Duplicate map keys are legal: any_encode collapses them.) */
static int any_skip2(rd_t *r, int depth, bool check_dups) {
  uint8_t tag;
  TRY(rd_u8(r, &tag));
  const uint8_t *s;
  uint32_t n32;
  uint64_t n;
  int64_t i64;
  switch (tag) {
  case 127: case 126: case 121: case 120: return 0;
  case 125: return rd_var_i64(r, &i64);
  case 124: return rd_exact(r, 4, &s);
  case 123: case 122: return rd_exact(r, 8, &s);
  case 119: case 116: return rd_buf(r, &s, &n32);
  case 118: { /* HashMap::with_capacity(len): (String, Any) = 48 bytes */
    TRY(rd_var_u64(r, &n));
    if (n && (n > (1ull << 40) || cap_to_buckets((size_t)n) * 49ull > ALLOC_LIMIT)) return YO_ERR_REFERENCE_PANIC;
    if (depth >= 64) return YO_ERR_UNSUPPORTED;
    for (uint64_t i = 0; i < n; i++) {
      TRY(rd_buf(r, &s, &n32));
      TRY(any_skip2(r, depth + 1, check_dups));
    }
    return 0;
  }
  case 117: /* Vec::with_capacity(len): Any = 24 bytes */
    TRY(rd_var_u64(r, &n));
    if (n > ALLOC_LIMIT / 24) return YO_ERR_REFERENCE_PANIC;
    if (depth >= 64) return YO_ERR_UNSUPPORTED;
    for (uint64_t i = 0; i < n; i++) TRY(any_skip2(r, depth + 1, check_dups));
    return 0;
  default: return YO_ERR_UNEXPECTED_VALUE;
  }
}
static int any_skip(upd_t *u, rd_t *r, int depth) { return any_skip2(r, depth, false); }

/* Any::encode number rules (any.rs:136-154) */
static void num_encode(wb_t *w, double x) {
  double t = trunc(x);
  if (t == x && t <= 9007199254740991.0 && t >= -9007199254740991.0) {
    wb_u8(w, 125);
    wb_var_i64(w, (int64_t)t);
  } else if ((double)(float)x == x) {
    float f = (float)x;
    uint32_t b;
    memcpy(&b, &f, 4);
    wb_u8(w, 124);
    for (int k = 3; k >= 0; k--) wb_u8(w, (uint8_t)(b >> (8 * k)));
  } else {
    uint64_t b;
    memcpy(&b, &x, 8);
    wb_u8(w, 123);
    for (int k = 7; k >= 0; k--) wb_u8(w, (uint8_t)(b >> (8 * k)));
  }
}
static void any_encode(rd_t *r, wb_t *w) {
  uint8_t tag = r->p[r->i++];
  const uint8_t *s = NULL;
  uint32_t n32;
  uint64_t n = 0;
  int64_t i64;
  switch (tag) {
  case 127: case 126: case 121: case 120: wb_u8(w, tag); return;
  case 125: rd_var_i64(r, &i64); num_encode(w, (double)i64); return;
  case 124: {
    rd_exact(r, 4, &s);
    uint32_t b = (uint32_t)s[0] << 24 | (uint32_t)s[1] << 16 | (uint32_t)s[2] << 8 | s[3];
    float f;
    memcpy(&f, &b, 4);
    num_encode(w, (double)f);
    return;
  }
  case 123: {
    rd_exact(r, 8, &s);
    uint64_t b = 0;
    for (int k = 0; k < 8; k++) b = b << 8 | s[k];
    double d;
    memcpy(&d, &b, 8);
    num_encode(w, d);
    return;
  }
  case 122: rd_exact(r, 8, &s); wb_u8(w, 122); wb_bytes(w, s, 8); return;
  case 119: case 116: rd_buf(r, &s, &n32); wb_u8(w, tag); wb_str(w, s, n32); return;
  case 117:
    rd_var_u64(r, &n);
    wb_u8(w, 117);
    wb_var(w, n);
    for (uint64_t i = 0; i < n; i++) any_encode(r, w);
    return;
  case 118: {
    rd_var_u64(r, &n);
    /* HashMap::insert (any.rs:61-68): a repeated key keeps its last value; RandomState
     * order policy: each distinct key is written where it occurs last */
    VEC(span_t) keys = {0};
    VEC(size_t) vals = {0};
    for (uint64_t i = 0; i < n; i++) {
      span_t k;
      rd_buf(r, &k.p, &k.n);
      size_t vpos = r->i;
      any_skip(NULL, r, 0);
      for (size_t j = 0; j < keys.n; j++)
        if (keys.d[j].n == k.n && !memcmp(keys.d[j].p, k.p, k.n)) {
          memmove(keys.d + j, keys.d + j + 1, (keys.n - j - 1) * sizeof(span_t));
          memmove(vals.d + j, vals.d + j + 1, (vals.n - j - 1) * sizeof(size_t));
          keys.n--;
          vals.n--;
          break;
        }
      VPUSH(keys, k);
      VPUSH(vals, vpos);
    }
    size_t end = r->i;
    wb_u8(w, 118);
    wb_var(w, keys.n);
    for (size_t j = 0; j < keys.n; j++) {
      wb_str(w, keys.d[j].p, keys.d[j].n);
      rd_t rv = {r->p, r->n, vals.d[j]};
      any_encode(&rv, w);
    }
    r->i = end;
    VFREE(keys);
    VFREE(vals);
    return;
  }
  }
}

/* ------------------------------------------------------------------ JSON (content refs 5/6)
 * ItemContent::Embed / Format carry JSON text (read_json -> Any::from_json, write_json ->
 * Any::to_json: yrs/src/updates/decoder.rs:175-178, encoder.rs:170-174, any.rs:185-198).
 * Restated here: serde_json 1.0.116's deserializer (Cargo.lock:725-726; default features,
 * i.e. no float_roundtrip / arbitrary_precision: parse_integer, parse_long_integer,
 * parse_decimal(+_overflow), parse_exponent(+_overflow), f64_from_parts with the POW10
 * table, parse_str escapes with paired-surrogate validation, recursion limit 128), yrs'
 * `Deserialize for Any` (yrs/src/encoding/serde/de.rs:17-211) with From<i64>/TryFrom<u64>
 * (yrs/src/any.rs:243-318), `Serialize for Any` (yrs/src/encoding/serde/ser.rs:16-54),
 * serde_json's CompactFormatter (string escapes, itoa) and ryu 1.0.17's shortest f64
 * (Cargo.lock:684-685) in its `format64` layout.  Every parse error is InvalidJSON.
 * Objects are a RandomState HashMap (de.rs:196-206): duplicate keys collapse (last value
 * wins) and the order of >= 2 distinct keys is random in yrs; policy: an entry is written
 * at the position of its key's LAST occurrence.  Parity: integers/strings/literals follow
 * the restated serde_json; floats are "parity unpinned" (no reference vector holds one),
 * the shortest-digit generator is pinned against CPython's repr (tests/test_json.py). */
typedef struct {
  const uint8_t *p;
  size_t n, i;
  int remaining_depth;
} jp_t;
static void jp_ws(jp_t *j) {
  while (j->i < j->n && (j->p[j->i] == ' ' || j->p[j->i] == '\n' || j->p[j->i] == '\t' || j->p[j->i] == '\r')) j->i++;
}
static int jp_peek(const jp_t *j) { return j->i < j->n ? j->p[j->i] : -1; }

/* --- unbounded-precision helpers for the shortest f64 digits (Burger & Dybvig free format,
 *     ties to even like ryu's d2d) */
#define BN_LIMBS 48
typedef struct {
  uint32_t w[BN_LIMBS];
} bn_t;
static void bn_set(bn_t *a, uint64_t v) {
  memset(a, 0, sizeof(*a));
  a->w[0] = (uint32_t)v;
  a->w[1] = (uint32_t)(v >> 32);
}
static void bn_mul_small(bn_t *a, uint32_t m) {
  uint64_t c = 0;
  for (int i = 0; i < BN_LIMBS; i++) {
    uint64_t t = (uint64_t)a->w[i] * m + c;
    a->w[i] = (uint32_t)t;
    c = t >> 32;
  }
}
static void bn_shl(bn_t *a, int k) {
  while (k >= 32) {
    memmove(a->w + 1, a->w, (BN_LIMBS - 1) * 4);
    a->w[0] = 0;
    k -= 32;
  }
  if (!k) return;
  for (int i = BN_LIMBS - 1; i > 0; i--) a->w[i] = a->w[i] << k | a->w[i - 1] >> (32 - k);
  a->w[0] <<= k;
}
static int bn_cmp(const bn_t *a, const bn_t *b) {
  for (int i = BN_LIMBS - 1; i >= 0; i--)
    if (a->w[i] != b->w[i]) return a->w[i] < b->w[i] ? -1 : 1;
  return 0;
}
static void bn_add(bn_t *r, const bn_t *a, const bn_t *b) {
  uint64_t c = 0;
  for (int i = 0; i < BN_LIMBS; i++) {
    uint64_t t = (uint64_t)a->w[i] + b->w[i] + c;
    r->w[i] = (uint32_t)t;
    c = t >> 32;
  }
}
static void bn_sub(bn_t *a, const bn_t *b) { /* a -= b, a >= b */
  int64_t br = 0;
  for (int i = 0; i < BN_LIMBS; i++) {
    int64_t t = (int64_t)a->w[i] - b->w[i] - br;
    br = t < 0;
    a->w[i] = (uint32_t)(t + (br ? (1ll << 32) : 0));
  }
}
/* shortest digits of a finite x > 0: digits[0..n), value = 0.d1..dn * 10^k */
static int f64_shortest(double x, char *digits, int *k_out) {
  uint64_t bits;
  memcpy(&bits, &x, 8);
  int be = (int)((bits >> 52) & 0x7FF);
  uint64_t f = bits & ((1ull << 52) - 1);
  int e;
  if (be == 0) e = -1074;
  else {
    f |= 1ull << 52;
    e = be - 1075;
  }
  const bool even = (f & 1) == 0;
  const bool unequal = be > 1 && f == (1ull << 52); /* lower gap is half the upper */
  bn_t r, s, mp, mm;
  if (e >= 0) {
    bn_set(&r, f);
    bn_shl(&r, e + (unequal ? 2 : 1));
    bn_set(&s, unequal ? 4 : 2);
    bn_set(&mp, 1);
    bn_shl(&mp, e + (unequal ? 1 : 0));
    bn_set(&mm, 1);
    bn_shl(&mm, e);
  } else {
    bn_set(&r, f);
    bn_shl(&r, unequal ? 2 : 1);
    bn_set(&s, 1);
    bn_shl(&s, -e + (unequal ? 2 : 1));
    bn_set(&mp, unequal ? 2 : 1);
    bn_set(&mm, 1);
  }
  int k = (int)ceil(log10(x) - 1e-10);
  if (k >= 0)
    for (int q = 0; q < k; q++) bn_mul_small(&s, 10);
  else
    for (int q = 0; q < -k; q++) {
      bn_mul_small(&r, 10);
      bn_mul_small(&mp, 10);
      bn_mul_small(&mm, 10);
    }
  bn_t hi;
  for (;;) { /* fixup: (r + m+) / s must be below 1 (<= 1 when the bound is inclusive) */
    bn_add(&hi, &r, &mp);
    int c = bn_cmp(&hi, &s);
    if (even ? c >= 0 : c > 0) {
      bn_mul_small(&s, 10);
      k++;
      continue;
    }
    bn_t hi10 = hi;
    bn_mul_small(&hi10, 10);
    c = bn_cmp(&hi10, &s);
    if (even ? c < 0 : c <= 0) {
      bn_mul_small(&r, 10);
      bn_mul_small(&mp, 10);
      bn_mul_small(&mm, 10);
      k--;
      continue;
    }
    break;
  }
  int n = 0;
  for (;;) {
    bn_mul_small(&r, 10);
    bn_mul_small(&mp, 10);
    bn_mul_small(&mm, 10);
    int d = 0;
    while (bn_cmp(&r, &s) >= 0) {
      bn_sub(&r, &s);
      d++;
    }
    int cl = bn_cmp(&r, &mm);
    bool tc1 = even ? cl <= 0 : cl < 0;
    bn_add(&hi, &r, &mp);
    int ch = bn_cmp(&hi, &s);
    bool tc2 = even ? ch >= 0 : ch > 0;
    if (!tc1 && !tc2) {
      digits[n++] = (char)('0' + d);
      continue;
    }
    if (tc1 && tc2) {
      bn_t r2 = r;
      bn_shl(&r2, 1);
      int c2 = bn_cmp(&r2, &s);
      if (c2 > 0 || (c2 == 0 && (d & 1))) d++;
    } else if (tc2)
      d++;
    digits[n++] = (char)('0' + d);
    break;
  }
  /* a rounded-up 9 carries (never produced for doubles; kept for safety) */
  for (int q = n - 1; q > 0 && digits[q] > '9'; q--) {
    digits[q] = '0';
    digits[q - 1]++;
  }
  if (digits[0] > '9') {
    digits[0] = '1';
    k++;
  }
  while (n > 1 && digits[n - 1] == '0') n--;
  *k_out = k;
  return n;
}
/* ryu::Buffer::format_finite (ryu/src/pretty/mod.rs format64) */
static void f64_ryu(wb_t *w, double x) {
  uint64_t bits;
  memcpy(&bits, &x, 8);
  if (bits >> 63) wb_u8(w, '-');
  if ((bits << 1) == 0) {
    wb_bytes(w, (const uint8_t *)"0.0", 3);
    return;
  }
  char dg[40];
  int kk;
  const int len = f64_shortest(fabs(x), dg, &kk);
  const int k = kk - len; /* value = digits * 10^k */
  if (0 <= k && kk <= 16) {
    wb_bytes(w, (const uint8_t *)dg, len);
    for (int i = len; i < kk; i++) wb_u8(w, '0');
    wb_bytes(w, (const uint8_t *)".0", 2);
  } else if (0 < kk && kk <= 16) {
    wb_bytes(w, (const uint8_t *)dg, kk);
    wb_u8(w, '.');
    wb_bytes(w, (const uint8_t *)dg + kk, len - kk);
  } else if (-5 < kk && kk <= 0) {
    wb_bytes(w, (const uint8_t *)"0.", 2);
    for (int i = 0; i < -kk; i++) wb_u8(w, '0');
    wb_bytes(w, (const uint8_t *)dg, len);
  } else {
    wb_u8(w, (uint8_t)dg[0]);
    if (len > 1) {
      wb_u8(w, '.');
      wb_bytes(w, (const uint8_t *)dg + 1, len - 1);
    }
    wb_u8(w, 'e');
    char eb[8];
    int en = snprintf(eb, sizeof eb, "%d", kk - 1);
    wb_bytes(w, (const uint8_t *)eb, en);
  }
}
static void wb_i64(wb_t *w, int64_t v) { /* itoa */
  char b[24];
  int n = snprintf(b, sizeof b, "%lld", (long long)v);
  wb_bytes(w, (const uint8_t *)b, n);
}
/* Serialize for Any, Number (ser.rs:25-34): `value as i64 as f64 == value` -> i64, else f64 */
static void json_number(wb_t *w, double x) {
  int64_t i;
  if (x != x) i = 0;
  else if (x >= 9223372036854775808.0) i = INT64_MAX; /* Rust `as` saturates */
  else if (x < -9223372036854775808.0) i = INT64_MIN;
  else i = (int64_t)x;
  if ((double)i == x) wb_i64(w, i);
  else if (isfinite(x)) f64_ryu(w, x);
  else wb_bytes(w, (const uint8_t *)"null", 4);
}
/* serde_json format_escaped_str: ", \ and control bytes; \u00XX in lowercase hex */
static void json_str_out(wb_t *w, const uint8_t *s, size_t n) {
  static const char hex[] = "0123456789abcdef";
  wb_u8(w, '"');
  for (size_t i = 0; i < n; i++) {
    uint8_t c = s[i];
    switch (c) {
    case '"': wb_bytes(w, (const uint8_t *)"\\\"", 2); break;
    case '\\': wb_bytes(w, (const uint8_t *)"\\\\", 2); break;
    case '\b': wb_bytes(w, (const uint8_t *)"\\b", 2); break;
    case '\f': wb_bytes(w, (const uint8_t *)"\\f", 2); break;
    case '\n': wb_bytes(w, (const uint8_t *)"\\n", 2); break;
    case '\r': wb_bytes(w, (const uint8_t *)"\\r", 2); break;
    case '\t': wb_bytes(w, (const uint8_t *)"\\t", 2); break;
    default:
      if (c < 0x20) {
        uint8_t e[6] = {'\\', 'u', '0', '0', (uint8_t)hex[c >> 4], (uint8_t)hex[c & 15]};
        wb_bytes(w, e, 6);
      } else
        wb_u8(w, c);
    }
  }
  wb_u8(w, '"');
}
static int hexval(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
static int jp_hex4(jp_t *j, uint32_t *v) {
  if (j->n - j->i < 4) return YO_ERR_INVALID_JSON;
  uint32_t x = 0;
  for (int q = 0; q < 4; q++) {
    int h = hexval(j->p[j->i + q]);
    if (h < 0) return YO_ERR_INVALID_JSON;
    x = x << 4 | (uint32_t)h;
  }
  j->i += 4;
  *v = x;
  return 0;
}
static void wb_utf8(wb_t *w, uint32_t c) {
  if (c < 0x80) wb_u8(w, (uint8_t)c);
  else if (c < 0x800) {
    wb_u8(w, (uint8_t)(0xC0 | c >> 6));
    wb_u8(w, (uint8_t)(0x80 | (c & 63)));
  } else if (c < 0x10000) {
    wb_u8(w, (uint8_t)(0xE0 | c >> 12));
    wb_u8(w, (uint8_t)(0x80 | ((c >> 6) & 63)));
    wb_u8(w, (uint8_t)(0x80 | (c & 63)));
  } else {
    wb_u8(w, (uint8_t)(0xF0 | c >> 18));
    wb_u8(w, (uint8_t)(0x80 | ((c >> 12) & 63)));
    wb_u8(w, (uint8_t)(0x80 | ((c >> 6) & 63)));
    wb_u8(w, (uint8_t)(0x80 | (c & 63)));
  }
}
/* serde_json parse_str (validate = true): the opening quote is consumed; unescaped bytes -> w */
static int jp_string(jp_t *j, wb_t *w) {
  for (;;) {
    if (j->i >= j->n) return YO_ERR_INVALID_JSON;
    uint8_t c = j->p[j->i++];
    if (c == '"') return 0;
    if (c < 0x20) return YO_ERR_INVALID_JSON;
    if (c != '\\') {
      wb_u8(w, c);
      continue;
    }
    if (j->i >= j->n) return YO_ERR_INVALID_JSON;
    c = j->p[j->i++];
    switch (c) {
    case '"': case '\\': case '/': wb_u8(w, c); break;
    case 'b': wb_u8(w, '\b'); break;
    case 'f': wb_u8(w, '\f'); break;
    case 'n': wb_u8(w, '\n'); break;
    case 'r': wb_u8(w, '\r'); break;
    case 't': wb_u8(w, '\t'); break;
    case 'u': {
      uint32_t n1;
      TRY(jp_hex4(j, &n1));
      if (n1 >= 0xDC00 && n1 <= 0xDFFF) return YO_ERR_INVALID_JSON;
      if (n1 >= 0xD800 && n1 <= 0xDBFF) {
        if (j->n - j->i < 2 || j->p[j->i] != '\\' || j->p[j->i + 1] != 'u') return YO_ERR_INVALID_JSON;
        j->i += 2;
        uint32_t n2;
        TRY(jp_hex4(j, &n2));
        if (n2 < 0xDC00 || n2 > 0xDFFF) return YO_ERR_INVALID_JSON;
        n1 = (((n1 - 0xD800) << 10) | (n2 - 0xDC00)) + 0x10000;
      }
      wb_utf8(w, n1);
      break;
    }
    default: return YO_ERR_INVALID_JSON;
    }
  }
}
static double pow10_tab(int e) { /* serde_json POW10[e], 0 <= e <= 308: correctly rounded 1e{e} */
  char b[16];
  snprintf(b, sizeof b, "1e%d", e);
  return strtod(b, NULL);
}
/* f64_from_parts (not float_roundtrip) */
static int f64_from_parts(bool positive, uint64_t significand, int64_t exponent, double *out) {
  double f = (double)significand;
  for (;;) {
    uint64_t ae = exponent < 0 ? (uint64_t)(-exponent) : (uint64_t)exponent;
    if (ae <= 308) {
      if (exponent >= 0) {
        f *= pow10_tab((int)ae);
        if (isinf(f)) return YO_ERR_INVALID_JSON;
      } else
        f /= pow10_tab((int)ae);
      break;
    }
    if (f == 0.0) break;
    if (exponent >= 0) return YO_ERR_INVALID_JSON;
    f /= 1e308;
    exponent += 308;
  }
  *out = positive ? f : -f;
  return 0;
}
#define OVERFLOW10(a, b, c) ((a) >= (c) / 10 && ((a) > (c) / 10 || (b) > (c) % 10))
static int jp_exponent(jp_t *j, bool positive, uint64_t sig, int64_t starting_exp, double *out) {
  j->i++; /* e / E */
  bool positive_exp = true;
  if (jp_peek(j) == '+') j->i++;
  else if (jp_peek(j) == '-') {
    j->i++;
    positive_exp = false;
  }
  int c = jp_peek(j);
  if (c < '0' || c > '9') return YO_ERR_INVALID_JSON;
  j->i++;
  int32_t exp = c - '0';
  while ((c = jp_peek(j)) >= '0' && c <= '9') {
    j->i++;
    int32_t d = c - '0';
    if (OVERFLOW10(exp, d, INT32_MAX)) { /* parse_exponent_overflow */
      if (sig != 0 && positive_exp) return YO_ERR_INVALID_JSON;
      while ((c = jp_peek(j)) >= '0' && c <= '9') j->i++;
      *out = positive ? 0.0 : -0.0;
      return 0;
    }
    exp = exp * 10 + d;
  }
  int64_t fe = positive_exp ? starting_exp + exp : starting_exp - exp; /* saturating_* on i32 */
  if (fe > INT32_MAX) fe = INT32_MAX;
  if (fe < INT32_MIN) fe = INT32_MIN;
  return f64_from_parts(positive, sig, fe, out);
}
static int jp_decimal(jp_t *j, bool positive, uint64_t sig, int64_t exp_before, double *out) {
  j->i++; /* '.' */
  int64_t after = 0;
  int c;
  while ((c = jp_peek(j)) >= '0' && c <= '9') {
    uint64_t d = (uint64_t)(c - '0');
    if (OVERFLOW10(sig, d, UINT64_MAX)) { /* parse_decimal_overflow: ignore further digits */
      while ((c = jp_peek(j)) >= '0' && c <= '9') j->i++;
      if (c == 'e' || c == 'E') return jp_exponent(j, positive, sig, exp_before + after, out);
      return f64_from_parts(positive, sig, exp_before + after, out);
    }
    j->i++;
    sig = sig * 10 + d;
    after--;
  }
  if (after == 0) return YO_ERR_INVALID_JSON;
  c = jp_peek(j);
  if (c == 'e' || c == 'E') return jp_exponent(j, positive, sig, exp_before + after, out);
  return f64_from_parts(positive, sig, exp_before + after, out);
}
/* deserialize_any on a number, then Deserialize for Any, then Serialize for Any */
static int jp_number(jp_t *j, bool positive, wb_t *w) {
  int c = jp_peek(j);
  if (c < '0' || c > '9') return YO_ERR_INVALID_JSON;
  j->i++;
  uint64_t sig = (uint64_t)(c - '0');
  double f;
  if (c == '0') {
    c = jp_peek(j);
    if (c >= '0' && c <= '9') return YO_ERR_INVALID_JSON; /* only one leading '0' */
  } else {
    while ((c = jp_peek(j)) >= '0' && c <= '9') {
      uint64_t d = (uint64_t)(c - '0');
      if (OVERFLOW10(sig, d, UINT64_MAX)) { /* parse_long_integer: further digits scale */
        int64_t exponent = 0;
        while ((c = jp_peek(j)) >= '0' && c <= '9') {
          j->i++;
          exponent++;
        }
        if (c == '.') TRY(jp_decimal(j, positive, sig, exponent, &f));
        else if (c == 'e' || c == 'E') TRY(jp_exponent(j, positive, sig, exponent, &f));
        else TRY(f64_from_parts(positive, sig, exponent, &f));
        json_number(w, f); /* visit_f64 -> Any::Number */
        return 0;
      }
      j->i++;
      sig = sig * 10 + d;
    }
  }
  c = jp_peek(j);
  if (c == '.') {
    TRY(jp_decimal(j, positive, sig, 0, &f));
    json_number(w, f);
    return 0;
  }
  if (c == 'e' || c == 'E') {
    TRY(jp_exponent(j, positive, sig, 0, &f));
    json_number(w, f);
    return 0;
  }
  if (positive) { /* visit_u64 -> TryFrom<u64> for Any (any.rs:302-318) */
    if (sig > (uint64_t)INT64_MAX) return YO_ERR_INVALID_JSON;
    double v = (double)sig;
    if (v <= 9007199254740991.0) json_number(w, v);
    else wb_i64(w, v >= 9223372036854775808.0 ? INT64_MAX : (int64_t)v); /* BigInt(v as f64 as i64) */
    return 0;
  }
  int64_t neg = (int64_t)(0 - sig); /* (significand as i64).wrapping_neg() */
  if (neg >= 0) {                   /* -0 or below i64::MIN: visit_f64(-(significand as f64)) */
    json_number(w, -(double)sig);
    return 0;
  }
  double v = (double)neg; /* visit_i64 -> From<i64> (impl_from_bigint) */
  if (v >= -9007199254740991.0) json_number(w, v);
  else wb_i64(w, neg);
  return 0;
}
typedef struct {
  wb_t key; /* unescaped key bytes */
  wb_t val; /* canonical value text */
} jent_t;
static int jp_value(jp_t *j, wb_t *w) {
  jp_ws(j);
  int c = jp_peek(j);
  switch (c) {
  case 'n': case 't': case 'f': {
    const char *lit = c == 'n' ? "null" : c == 't' ? "true" : "false";
    size_t ln = strlen(lit);
    if (j->n - j->i < ln || memcmp(j->p + j->i, lit, ln)) return YO_ERR_INVALID_JSON;
    j->i += ln;
    wb_bytes(w, (const uint8_t *)lit, ln);
    return 0;
  }
  case '-': j->i++; return jp_number(j, false, w);
  case '"': {
    j->i++;
    wb_t s = {0};
    int e = jp_string(j, &s);
    if (!e) json_str_out(w, s.d, s.n);
    VFREE(s);
    return e;
  }
  case '[': {
    if (--j->remaining_depth == 0) return YO_ERR_INVALID_JSON;
    j->i++;
    wb_u8(w, '[');
    jp_ws(j);
    if (jp_peek(j) == ']') j->i++;
    else
      for (bool first = true;; first = false) {
        if (!first) wb_u8(w, ',');
        TRY(jp_value(j, w));
        jp_ws(j);
        c = jp_peek(j);
        if (c == ']') {
          j->i++;
          break;
        }
        if (c != ',') return YO_ERR_INVALID_JSON;
        j->i++;
        jp_ws(j);
        if (jp_peek(j) == ']') return YO_ERR_INVALID_JSON; /* trailing comma */
      }
    wb_u8(w, ']');
    j->remaining_depth++;
    return 0;
  }
  case '{': {
    if (--j->remaining_depth == 0) return YO_ERR_INVALID_JSON;
    j->i++;
    VEC(jent_t) es = {0};
    int err = 0;
    jp_ws(j);
    if (jp_peek(j) == '}') j->i++;
    else
      for (;;) {
        jp_ws(j);
        if (jp_peek(j) != '"') {
          err = YO_ERR_INVALID_JSON;
          break;
        }
        j->i++;
        jent_t e = {{0}, {0}};
        VPUSH(es, e);
        jent_t *cur = &es.d[es.n - 1];
        if ((err = jp_string(j, &cur->key))) break;
        jp_ws(j);
        if (jp_peek(j) != ':') {
          err = YO_ERR_INVALID_JSON;
          break;
        }
        j->i++;
        if ((err = jp_value(j, &cur->val))) break;
        jp_ws(j);
        c = jp_peek(j);
        if (c == '}') {
          j->i++;
          break;
        }
        if (c != ',') {
          err = YO_ERR_INVALID_JSON;
          break;
        }
        j->i++;
        jp_ws(j);
        if (jp_peek(j) == '}') {
          err = YO_ERR_INVALID_JSON; /* trailing comma */
          break;
        }
      }
    if (!err) {
      wb_u8(w, '{');
      bool first = true;
      for (size_t a = 0; a < es.n; a++) {
        bool later = false;
        for (size_t b = a + 1; b < es.n && !later; b++)
          later = es.d[b].key.n == es.d[a].key.n && !memcmp(es.d[b].key.d, es.d[a].key.d, es.d[a].key.n);
        if (later) continue; /* HashMap::insert: the last value of a key survives */
        if (!first) wb_u8(w, ',');
        first = false;
        json_str_out(w, es.d[a].key.d, es.d[a].key.n);
        wb_u8(w, ':');
        wb_bytes(w, es.d[a].val.d, es.d[a].val.n);
      }
      wb_u8(w, '}');
      j->remaining_depth++;
    }
    for (size_t a = 0; a < es.n; a++) {
      VFREE(es.d[a].key);
      VFREE(es.d[a].val);
    }
    VFREE(es);
    return err;
  }
  default:
    if (c >= '0' && c <= '9') return jp_number(j, true, w);
    return YO_ERR_INVALID_JSON;
  }
}
/* serde_json::from_str::<Any>(src) then Any::to_json: canonical text into w, or InvalidJSON */
static int json_canon(const uint8_t *s, size_t n, wb_t *w) {
  jp_t j = {s, n, 0, 128};
  TRY(jp_value(&j, w));
  jp_ws(&j);
  return j.i == j.n ? 0 : YO_ERR_INVALID_JSON; /* TrailingCharacters */
}
/* test hooks: canonical JSON text, and ryu's format of one f64 */
int yo_json_canon(const uint8_t *s, size_t n, uint8_t **out, size_t *out_len) {
  wb_t w = {0};
  int e = json_canon(s, n, &w);
  if (e) {
    VFREE(w);
    return e;
  }
  wb_u8(&w, 0);
  *out = w.d;
  *out_len = w.n - 1;
  return 0;
}
int yo_f64_ryu(double x, char *buf, size_t cap) {
  wb_t w = {0};
  f64_ryu(&w, x);
  size_t n = w.n < cap - 1 ? w.n : cap - 1;
  memcpy(buf, w.d, n);
  buf[n] = 0;
  VFREE(w);
  return (int)n;
}

/* ------------------------------------------------------------------ content decode (block.rs:1786-1835) */
static int doc_options_any(upd_t *u, rd_t *r, blk_t *b);
static int doc_options_decode(upd_t *u, rd_t *r, blk_t *b) {
  /* Options::decode (doc.rs:840-872) */
  TRY(rd_buf(r, &b->cs.p, &b->cs.n)); /* guid */
  return doc_options_any(u, r, b);
}
/* the options Any that follows the guid */
static int doc_options_any(upd_t *u, rd_t *r, blk_t *b) {
  b->doc_skip_gc = 0;
  b->doc_auto_load = 0;
  b->doc_has_cid = 0;
  b->doc_enc_bytes = 1;
  size_t start = r->i;
  TRY(any_skip(u, r, 0));
  rd_t a = {r->p, r->n, start};
  if (a.p[a.i] != 118) return 0;
  a.i++;
  uint64_t n = 0;
  rd_var_u64(&a, &n);
  /* dedupe: last value wins per key; then apply each distinct key */
  VEC(span_t) keys = {0};
  VEC(size_t) vals = {0};
  for (uint64_t i = 0; i < n; i++) {
    span_t k;
    rd_buf(&a, &k.p, &k.n);
    size_t vpos = a.i;
    any_skip(u, &a, 0);
    size_t j = 0;
    for (; j < keys.n; j++)
      if (keys.d[j].n == k.n && !memcmp(keys.d[j].p, k.p, k.n)) break;
    if (j == keys.n) {
      VPUSH(keys, k);
      VPUSH(vals, vpos);
    } else
      vals.d[j] = vpos;
  }
  for (size_t j = 0; j < keys.n; j++) {
    const uint8_t *v = a.p + vals.d[j];
    span_t k = keys.d[j];
#define KEQ(lit) (k.n == sizeof(lit) - 1 && !memcmp(k.p, lit, k.n))
    if (KEQ("gc") && (v[0] == 120 || v[0] == 121)) b->doc_skip_gc = v[0] == 121;
    else if (KEQ("autoLoad") && (v[0] == 120 || v[0] == 121)) b->doc_auto_load = v[0] == 120;
    else if (KEQ("collectionId") && v[0] == 119) {
      rd_t sr = {a.p, a.n, vals.d[j] + 1};
      rd_buf(&sr, &b->doc_cid.p, &b->doc_cid.n);
      b->doc_has_cid = 1;
    } else if (KEQ("encoding")) {
      static const uint8_t one[8] = {0, 0, 0, 0, 0, 0, 0, 1};
      b->doc_enc_bytes = (v[0] == 122 && !memcmp(v + 1, one, 8));
    }
#undef KEQ
  }
  VFREE(keys);
  VFREE(vals);
  return 0;
}

static int content_decode(upd_t *u, rd_t *r, uint8_t ref, blk_t *b) {
  uint32_t n32;
  switch (ref) {
  case 1: TRY(rd_var_u32(r, &b->n)); b->len = b->n; return 0;
  case 2: { /* JSON: remaining = read_len as i32; reads remaining+1 strings */
    TRY(rd_var_u32(r, &n32));
    int32_t remaining = (int32_t)n32;
    if (remaining < 0) return YO_ERR_NOT_ENOUGH_MEMORY;
    b->e0 = (uint32_t)u->elems.n;
    b->n = 0;
    while (remaining >= 0) {
      span_t s;
      TRY(rd_buf(r, &s.p, &s.n));
      VPUSH(u->elems, s);
      b->n++;
      remaining--;
    }
    b->len = b->n;
    return 0;
  }
  case 3: TRY(rd_buf(r, &b->cs.p, &b->cs.n)); b->len = 1; return 0;
  case 4: TRY(rd_buf(r, &b->cs.p, &b->cs.n)); b->len = str_len16(b->cs.p, b->cs.n); return 0;
  case 5: case 6: { /* read_json (decoder.rs:175-178): serde_json parse at decode time */
    TRY(rd_buf(r, &b->cs.p, &b->cs.n));
    span_t js = b->cs;
    if (ref == 6) {
      TRY(rd_buf(r, &b->cs2.p, &b->cs2.n));
      js = b->cs2;
    }
    wb_t t = {0};
    int e = json_canon(js.p, js.n, &t);
    VFREE(t);
    b->len = 1;
    return e;
  }
  case 7: { /* TypeRef::decode (types/mod.rs:160-200), weak feature on (yffi) */
    TRY(rd_u8(r, &b->tref));
    b->len = 1;
    switch (b->tref) {
    case 0: case 1: case 2: case 4: case 5: case 6: case 9: case 15: return 0;
    case 3: return rd_buf(r, &b->cs.p, &b->cs.n);
    case 7: {
      uint8_t f;
      TRY(rd_u8(r, &f));
      b->mflags = f;
      TRY(rd_var_u64(r, &b->sc));
      TRY(rd_var_u32(r, &b->sk));
      if (f & 1) {
        TRY(rd_var_u64(r, &b->ec));
        TRY(rd_var_u32(r, &b->ek));
      } else {
        b->ec = b->sc;
        b->ek = b->sk;
      }
      return 0;
    }
    default: return YO_ERR_UNEXPECTED_VALUE;
    }
  }
  case 8: {
    TRY(rd_var_u32(r, &b->n));
    if ((uint64_t)b->n * 24 > ALLOC_LIMIT) return YO_ERR_NOT_ENOUGH_MEMORY;
    b->e0 = (uint32_t)u->elems.n;
    for (uint32_t i = 0; i < b->n; i++) {
      span_t s;
      s.p = r->p + r->i;
      size_t st = r->i;
      TRY(any_skip2(r, 0, true));
      s.n = (uint32_t)(r->i - st);
      VPUSH(u->elems, s);
    }
    b->len = b->n;
    return 0;
  }
  case 9: TRY(doc_options_decode(u, r, b)); b->len = 1; return 0;
  case 11: { /* Move::decode (moving.rs:306-333): flags read as i32 */
    int64_t f;
    TRY(rd_var_i64(r, &f));
    if (f < INT32_MIN || f > INT32_MAX) return YO_ERR_VAR_INT;
    b->mflags = f;
    TRY(rd_var_u64(r, &b->sc));
    TRY(rd_var_u32(r, &b->sk));
    if (!(f & 1)) {
      TRY(rd_var_u64(r, &b->ec));
      TRY(rd_var_u32(r, &b->ek));
    } else {
      b->ec = b->sc;
      b->ek = b->sk;
    }
    b->len = 1;
    return 0;
  }
  default: return YO_ERR_UNEXPECTED_VALUE;
  }
}

/* Update::decode_block (update.rs:433-488) */
static int decode_block(upd_t *u, rd_t *r, uint64_t client, uint32_t clock, blk_t *b, bool *has) {
  memset(b, 0, sizeof(*b));
  b->client = client;
  b->clock = clock;
  uint8_t info;
  TRY(rd_u8(r, &info));
  *has = true;
  if (info == 10) {
    b->kind = BK_SKIP;
    return rd_var_u32(r, &b->len);
  }
  if (info == 0) {
    b->kind = BK_GC;
    return rd_var_u32(r, &b->len);
  }
  b->kind = BK_ITEM;
  bool cant_copy = (info & 0xC0) == 0;
  uint32_t c32;
  if (info & 0x80) {
    TRY(rd_var_u32(r, &c32));
    b->oc = c32;
    TRY(rd_var_u32(r, &b->ok));
    b->has_origin = 1;
  }
  if (info & 0x40) {
    TRY(rd_var_u32(r, &c32));
    b->rc = c32;
    TRY(rd_var_u32(r, &b->rk));
    b->has_ro = 1;
  }
  if (cant_copy) {
    uint32_t pi;
    TRY(rd_var_u32(r, &pi));
    if (pi == 1) {
      b->pkind = PK_NAMED;
      TRY(rd_buf(r, &b->pname.p, &b->pname.n));
    } else {
      b->pkind = PK_ID;
      TRY(rd_var_u32(r, &c32));
      b->pc = c32;
      TRY(rd_var_u32(r, &b->pk));
    }
    if (info & 0x20) {
      b->has_psub = 1;
      TRY(rd_buf(r, &b->psub.p, &b->psub.n));
    }
  }
  b->ref = info & 15;
  TRY(content_decode(u, r, b->ref, b));
  if (b->len == 0) *has = false; /* Item::new -> None (block.rs:1225-1228) */
  return 0;
}

/* IdRange::decode (id_set.rs:268-286) */
static int idr_decode(rd_t *r, idr_t *out) {
  memset(out, 0, sizeof(*out));
  uint32_t n;
  TRY(rd_var_u32(r, &n));
  if (n == 1) {
    uint32_t c, l;
    TRY(rd_var_u32(r, &c));
    TRY(rd_var_u32(r, &l));
    if ((uint64_t)c + l > UINT32_MAX) return YO_ERR_REFERENCE_PANIC;
    out->cont = 1;
    out->c.s = c;
    out->c.e = c + l;
    return 0;
  }
  out->cont = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t c, l;
    TRY(rd_var_u32(r, &c));
    TRY(rd_var_u32(r, &l));
    if ((uint64_t)c + l > UINT32_MAX) return YO_ERR_REFERENCE_PANIC;
    rng_t g = {c, c + l};
    VPUSH(out->v, g);
  }
  return 0;
}

/* Decode for Update (update.rs:714-749) + DeleteSet::decode (id_set.rs:412-426) */
static int decode_update(upd_t *u, const uint8_t *p, size_t n) {
  memset(u, 0, sizeof(*u));
  u->base = p;
  u->len = n;
  rd_t r = {p, n, 0};
  uint32_t ncl;
  TRY(rd_var_u32(&r, &ncl));
  /* try_reserve(clients_len): (u64, VecDeque) = 40 bytes */
  TRY(hb_reserve(&u->clients, ncl, 40, true));
  for (uint32_t i = 0; i < ncl; i++) {
    uint32_t nb, c32, clock;
    TRY(rd_var_u32(&r, &nb));
    TRY(rd_var_u32(&r, &c32));
    TRY(rd_var_u32(&r, &clock));
    bool existed;
    int32_t e = hb_entry(&u->clients, c32, &existed);
    if (!existed) {
      blist_t bl = {0};
      VPUSH(u->lists, bl);
    }
    if (((uint64_t)u->lists.d[e].idx.n + nb) * 32 > ALLOC_LIMIT) return YO_ERR_NOT_ENOUGH_MEMORY;
    for (uint32_t j = 0; j < nb; j++) {
      blk_t b;
      bool has;
      TRY(decode_block(u, &r, c32, clock, &b, &has));
      if (has) {
        if ((uint64_t)clock + b.len > UINT32_MAX) return YO_ERR_REFERENCE_PANIC;
        clock += b.len;
        if (b.unsupported) u->unsupported = 1;
        VPUSH(u->blocks, b);
        VPUSH(u->lists.d[e].idx, (uint32_t)(u->blocks.n - 1));
      }
    }
  }
  uint32_t nds;
  TRY(rd_var_u32(&r, &nds));
  for (uint32_t i = 0; i < nds; i++) {
    uint32_t c32;
    TRY(rd_var_u32(&r, &c32));
    idr_t g;
    int e = idr_decode(&r, &g);
    if (e) {
      idr_free(&g);
      return e;
    }
    bool existed;
    int32_t k = hb_insert(&u->ds, c32, &existed);
    if (existed) {
      idr_free(&u->dsv.d[k]);
      u->dsv.d[k] = g;
    } else
      VPUSH(u->dsv, g);
  }
  return 0;
}

/* ------------------------------------------------------------------ IdRange ops (id_set.rs:104-247) */
static bool rng_disjoint(rng_t a, rng_t b) { return a.s > b.e || b.s > a.e; }
static void stable_sort_rng(rng_t *v, size_t n) { /* stable: merge sort by start */
  if (n < 2) return;
  rng_t *tmp = malloc(n * sizeof(rng_t));
  for (size_t w = 1; w < n; w *= 2) {
    for (size_t lo = 0; lo < n; lo += 2 * w) {
      size_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
      size_t i = lo, j = mid, k = lo;
      while (i < mid && j < hi) tmp[k++] = (v[j].s < v[i].s) ? v[j++] : v[i++];
      while (i < mid) tmp[k++] = v[i++];
      while (j < hi) tmp[k++] = v[j++];
    }
    memcpy(v, tmp, n * sizeof(rng_t));
  }
  free(tmp);
}
static void idr_squash(idr_t *r) {
  if (r->cont || r->v.n == 0) return;
  rng_t *v = r->v.d;
  size_t len = r->v.n;
  stable_sort_rng(v, len);
  size_t new_len = 1, cur = 0;
  for (size_t i = 1; i < len; i++) {
    rng_t nx = v[i];
    if (!rng_disjoint(v[cur], nx)) {
      if (nx.s < v[cur].s) v[cur].s = nx.s;
      if (nx.e > v[cur].e) v[cur].e = nx.e;
    } else {
      cur = new_len;
      v[cur] = nx;
      new_len++;
    }
  }
  if (new_len == 1) {
    r->cont = 1;
    r->c = v[0];
    VFREE(r->v);
  } else
    r->v.n = new_len;
}
static bool idr_is_squashed(const idr_t *r) {
  if (r->cont) return true;
  for (size_t i = 1; i < r->v.n; i++)
    if (r->v.d[i].s < r->v.d[i - 1].e) return false;
  return true;
}
static void idr_clone(idr_t *dst, const idr_t *src) {
  memset(dst, 0, sizeof(*dst));
  dst->cont = src->cont;
  dst->c = src->c;
  for (size_t i = 0; i < src->v.n; i++) VPUSH(dst->v, src->v.d[i]);
}
/* IdRange::merge (id_set.rs:189-216) */
static void idr_merge(idr_t *a, const idr_t *b) {
  if (a->cont && b->cont) {
    bool never = a->c.e < b->c.s || b->c.e < a->c.s;
    if (never) {
      rng_t x = a->c;
      a->cont = 0;
      a->v.n = 0;
      VPUSH(a->v, x);
      VPUSH(a->v, b->c);
    } else {
      if (b->c.s < a->c.s) a->c.s = b->c.s;
      if (b->c.e > a->c.e) a->c.e = b->c.e;
    }
  } else if (!a->cont && b->cont) {
    VPUSH(a->v, b->c);
  } else if (a->cont && !b->cont) {
    rng_t x = a->c;
    a->cont = 0;
    a->v.n = 0;
    for (size_t i = 0; i < b->v.n; i++) VPUSH(a->v, b->v.d[i]);
    VPUSH(a->v, x);
  } else {
    for (size_t i = 0; i < b->v.n; i++) VPUSH(a->v, b->v.d[i]);
  }
}
static void idr_encode_raw(wb_t *w, const idr_t *r) {
  if (r->cont) {
    wb_var(w, 1);
    wb_var(w, r->c.s);
    wb_var(w, (uint32_t)(r->c.e - r->c.s));
  } else {
    wb_var(w, (uint32_t)r->v.n);
    for (size_t i = 0; i < r->v.n; i++) {
      wb_var(w, r->v.d[i].s);
      wb_var(w, (uint32_t)(r->v.d[i].e - r->v.d[i].s));
    }
  }
}
static void idr_encode(wb_t *w, const idr_t *r) {
  if (idr_is_squashed(r)) {
    idr_encode_raw(w, r);
  } else {
    idr_t c;
    idr_clone(&c, r);
    idr_squash(&c);
    idr_encode_raw(w, &c);
    idr_free(&c);
  }
}
/* IdSet::encode (id_set.rs:401-410) */
static void ds_encode(wb_t *w, const hb_t *t, const idr_t *vals) {
  wb_var(w, (uint32_t)t->items);
  int32_t *ord = malloc((t->items + 1) * sizeof(int32_t));
  size_t k = hb_order(t, ord);
  for (size_t i = 0; i < k; i++) {
    wb_var(w, t->keys.d[ord[i]]);
    idr_encode(w, &vals[ord[i]]);
  }
  free(ord);
}

/* ------------------------------------------------------------------ block encode (slice.rs:199-251, block.rs:1711-1754) */
typedef struct {
  const blk_t *b; /* original decoded block (NULL for synthesized Skip) */
  uint32_t off;   /* ItemSlice start / GC slice offset */
  uint64_t client;
  uint32_t clock, len;
  uint8_t kind;
} car_t;

static int encode_item(wb_t *w, const upd_t *u, const blk_t *b, uint32_t off) {
  uint8_t info = (b->has_origin ? 0x80 : 0) | (b->has_ro ? 0x40 : 0) | (b->has_psub ? 0x20 : 0) | (b->ref & 15);
  bool origin = b->has_origin;
  uint64_t oc = b->oc;
  uint32_t ok = b->ok;
  if (off != 0) {
    origin = true;
    oc = b->client;
    ok = b->clock + off - 1;
    info |= 0x80;
  }
  bool cant_copy = (info & 0xC0) == 0;
  wb_u8(w, info);
  if (origin) {
    wb_var(w, oc);
    wb_var(w, ok);
  }
  if (b->has_ro) {
    wb_var(w, b->rc);
    wb_var(w, b->rk);
  }
  if (cant_copy) {
    if (b->pkind == PK_NAMED) {
      wb_var(w, 1);
      wb_str(w, b->pname.p, b->pname.n);
    } else if (b->pkind == PK_ID) {
      wb_var(w, 0);
      wb_var(w, b->pc);
      wb_var(w, b->pk);
    } else
      return YO_ERR_REFERENCE_PANIC;
    if (b->has_psub) wb_str(w, b->psub.p, b->psub.n);
  }
  uint32_t end = b->len - 1; /* ItemSlice::new(ptr, offset, len - 1) */
  switch (b->ref) {
  case 1: wb_var(w, (uint32_t)(end - off + 1)); return 0;
  case 2:
    wb_var(w, (uint32_t)(end - off + 1));
    for (uint32_t i = off; i <= end && i < b->n; i++) wb_str(w, u->elems.d[b->e0 + i].p, u->elems.d[b->e0 + i].n);
    return 0;
  case 3: wb_str(w, b->cs.p, b->cs.n); return 0;
  case 4: {
    const uint8_t *s = b->cs.p;
    uint32_t n = b->cs.n, bo;
    if (off != 0) {
      TRY(str_split16(s, n, off, &bo));
      s += bo;
      n -= bo;
    }
    if (end != 0) {
      TRY(str_split16(s, n, (uint32_t)(end - off + 1), &bo));
      n = bo;
    }
    wb_str(w, s, n);
    return 0;
  }
  case 5: /* ItemContent::Embed: write_json (encoder.rs:170-174) */
  case 6: { /* ItemContent::Format: write_key + write_json */
    if (b->ref == 6) wb_str(w, b->cs.p, b->cs.n);
    const span_t js = b->ref == 6 ? b->cs2 : b->cs;
    wb_t t = {0};
    int e = json_canon(js.p, js.n, &t);
    if (!e) wb_str(w, t.d, (uint32_t)t.n);
    VFREE(t);
    return e;
  }
  case 7:
    wb_u8(w, b->tref);
    if (b->tref == 3) wb_str(w, b->cs.p, b->cs.n);
    if (b->tref == 7) { /* TypeRef::WeakLink encode (types/mod.rs:134-156) */
      bool single = b->sc == b->ec && b->sk == b->ek;
      wb_u8(w, (uint8_t)((single ? 0 : 1) | (b->mflags & 2) | (b->mflags & 4)));
      wb_var(w, b->sc);
      wb_var(w, b->sk);
      if (!single) {
        wb_var(w, b->ec);
        wb_var(w, b->ek);
      }
    }
    return 0;
  case 8:
    wb_var(w, (uint32_t)(end - off + 1));
    for (uint32_t i = off; i <= end && i < b->n; i++) {
      rd_t r = {u->elems.d[b->e0 + i].p, u->elems.d[b->e0 + i].n, 0};
      any_encode(&r, w);
    }
    return 0;
  case 9: { /* Options::encode (doc.rs:832-838); map order = as_any insertion order (policy) */
    wb_str(w, b->cs.p, b->cs.n);
    wb_u8(w, 118);
    wb_var(w, b->doc_has_cid ? 5 : 4);
    wb_str(w, (const uint8_t *)"gc", 2);
    wb_u8(w, b->doc_skip_gc ? 121 : 120);
    if (b->doc_has_cid) {
      wb_str(w, (const uint8_t *)"collectionId", 12);
      wb_u8(w, 119);
      wb_str(w, b->doc_cid.p, b->doc_cid.n);
    }
    wb_str(w, (const uint8_t *)"encoding", 8);
    wb_u8(w, 122);
    for (int k = 0; k < 7; k++) wb_u8(w, 0);
    wb_u8(w, b->doc_enc_bytes ? 1 : 0);
    wb_str(w, (const uint8_t *)"autoLoad", 8);
    wb_u8(w, b->doc_auto_load ? 120 : 121);
    wb_str(w, (const uint8_t *)"shouldLoad", 10);
    wb_u8(w, b->doc_auto_load ? 120 : 121); /* should_load = should_load(false) || auto_load */
    return 0;
  }
  case 11: { /* Move::encode (moving.rs:277-304) */
    bool collapsed = b->sc == b->ec && b->sk == b->ek;
    int32_t fl = (int32_t)b->mflags;
    int32_t prio = fl >> 6;
    int32_t bb = (collapsed ? 1 : 0) | ((fl & 2) ? 2 : 0) | ((fl & 4) ? 4 : 0);
    bb |= (int32_t)((uint32_t)prio << 6);
    wb_var_i64(w, bb);
    wb_var(w, b->sc);
    wb_var(w, b->sk);
    if (!collapsed) {
      wb_var(w, b->ec);
      wb_var(w, b->ek);
    }
    return 0;
  }
  }
  return YO_ERR_REFERENCE_PANIC;
}
/* BlockCarrier::encode_with_offset (update.rs:886-901) */
static int encode_carrier(wb_t *w, const upd_t *u, const car_t *c, uint32_t offset) {
  if (c->kind == BK_SKIP) {
    wb_u8(w, 10);
    wb_var(w, (uint32_t)(c->len - offset));
    return 0;
  }
  if (c->kind == BK_GC) {
    wb_u8(w, 0);
    wb_var(w, (uint32_t)(c->len - offset));
    return 0;
  }
  return encode_item(w, u, c->b, c->off + offset);
}

/* ------------------------------------------------------------------ encode_diff (update.rs:490-535) */
typedef struct {
  uint64_t client;
  VEC(car_t) cars;
  VEC(const upd_t *) ups;
} clist_t;
/* sv_get: returns remote clock for client */
typedef struct {
  hb_t t;
  VEC(uint32_t) clocks;
} sv_t;
static uint32_t sv_get(const sv_t *sv, uint64_t client) {
  if (!sv) return 0;
  int32_t e = hb_find(&sv->t, client);
  return e >= 0 ? sv->clocks.d[e] : 0;
}
static int encode_blocks(wb_t *w, clist_t *cl, size_t ncl, const sv_t *sv) {
  /* per client: drop leading Skips and blocks ending at/below the remote clock */
  typedef struct {
    uint64_t client;
    uint32_t offset;
    size_t first, ci;
  } sel_t;
  sel_t *sel = malloc((ncl + 1) * sizeof(sel_t));
  size_t ns = 0;
  for (size_t i = 0; i < ncl; i++) {
    uint32_t remote = sv_get(sv, cl[i].client);
    for (size_t k = 0; k < cl[i].cars.n; k++) {
      car_t *c = &cl[i].cars.d[k];
      if (c->kind == BK_SKIP) continue;
      if ((uint32_t)(c->clock + c->len) > remote) {
        int64_t o = (int64_t)remote - (int64_t)c->clock;
        sel[ns].client = cl[i].client;
        sel[ns].offset = o > 0 ? (uint32_t)o : 0;
        sel[ns].first = k;
        sel[ns].ci = i;
        ns++;
        break;
      }
    }
  }
  /* sort by client desc */
  for (size_t i = 1; i < ns; i++) {
    sel_t t = sel[i];
    size_t j = i;
    while (j > 0 && sel[j - 1].client < t.client) {
      sel[j] = sel[j - 1];
      j--;
    }
    sel[j] = t;
  }
  wb_var(w, ns);
  for (size_t s = 0; s < ns; s++) {
    clist_t *c = &cl[sel[s].ci];
    size_t cnt = c->cars.n - sel[s].first;
    wb_var(w, cnt);
    wb_var(w, c->client);
    car_t *f = &c->cars.d[sel[s].first];
    wb_var(w, (uint32_t)(f->clock + sel[s].offset));
    for (size_t k = sel[s].first; k < c->cars.n; k++) {
      int e = encode_carrier(w, c->ups.d[k], &c->cars.d[k], k == sel[s].first ? sel[s].offset : 0);
      if (e) {
        free(sel);
        return e;
      }
    }
  }
  free(sel);
  return 0;
}

/* ------------------------------------------------------------------ merge (update.rs:537-704) */
typedef struct {
  const upd_t *u;
  uint32_t *stream; /* block indices, clients desc, Skips dropped (update.rs:1031-1057) */
  size_t n, pos;
  int has;
  car_t cur;
  int64_t t;   /* heap mode: iteration of last re-insert (-1 never) */
  size_t idx;  /* input order */
} dec_t;

static car_t car_of(const blk_t *b) {
  car_t c = {b, 0, b->client, b->clock, b->len, b->kind};
  return c;
}
static void dec_next(dec_t *d) {
  if (d->pos < d->n) {
    d->cur = car_of(&d->u->blocks.d[d->stream[d->pos++]]);
    d->has = 1;
  } else
    d->has = 0;
}
static int cmp_u64_desc(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? 1 : x > y ? -1 : 0;
}
static void dec_init(dec_t *d, const upd_t *u, size_t idx) {
  memset(d, 0, sizeof(*d));
  d->u = u;
  d->idx = idx;
  d->t = -1;
  size_t nk = u->clients.keys.n;
  uint64_t *ks = malloc((nk + 1) * sizeof(uint64_t));
  for (size_t i = 0; i < nk; i++) ks[i] = u->clients.keys.d[i];
  qsort(ks, nk, sizeof(uint64_t), cmp_u64_desc);
  d->stream = malloc((u->blocks.n + 1) * sizeof(uint32_t));
  for (size_t i = 0; i < nk; i++) {
    int32_t e = hb_find(&u->clients, ks[i]);
    for (size_t k = 0; k < u->lists.d[e].idx.n; k++) {
      uint32_t bi = u->lists.d[e].idx.d[k];
      if (u->blocks.d[bi].kind != BK_SKIP) d->stream[d->n++] = bi;
    }
  }
  free(ks);
  dec_next(d);
}
/* comparator of update.rs:572-589 (Skips never reach it: ignore_skip) */
static bool dec_less(const dec_t *a, const dec_t *b) {
  const car_t *l = &a->cur, *r = &b->cur;
  if (l->client != r->client) return l->client > r->client;
  if (l->clock == r->clock) return l->kind != r->kind; /* Equal if same type, else Less */
  return l->clock < r->clock;
}
/* the same with the Item-vs-GC tie read as Equal: a consistent order (policy above 20) */
static bool key_less(const dec_t *a, const dec_t *b) {
  const car_t *l = &a->cur, *r = &b->cur;
  if (l->client != r->client) return l->client > r->client;
  return l->clock < r->clock;
}
static bool heap_less(const dec_t *a, const dec_t *b) {
  const car_t *l = &a->cur, *r = &b->cur;
  if (l->client != r->client) return l->client > r->client;
  if (l->clock != r->clock) return l->clock < r->clock;
  if (a->t != b->t) return a->t > b->t;
  return a->idx < b->idx;
}
static void heap_push(dec_t **h, size_t *n, dec_t *d) {
  size_t i = (*n)++;
  h[i] = d;
  while (i > 0) {
    size_t p = (i - 1) / 2;
    if (!heap_less(h[i], h[p])) break;
    dec_t *t = h[i];
    h[i] = h[p];
    h[p] = t;
    i = p;
  }
}
static dec_t *heap_pop(dec_t **h, size_t *n) {
  dec_t *top = h[0];
  h[0] = h[--(*n)];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < *n && heap_less(h[l], h[m])) m = l;
    if (r < *n && heap_less(h[r], h[m])) m = r;
    if (m == i) break;
    dec_t *t = h[i];
    h[i] = h[m];
    h[m] = t;
    i = m;
  }
  return top;
}

/* BlockCarrier::splice (update.rs:795-816; block.rs:435-478, 1837-1879) */
static int car_splice(const car_t *c, uint32_t offset, car_t *out) {
  *out = *c;
  if (c->kind == BK_GC || c->kind == BK_SKIP) {
    out->clock = c->clock + offset;
    out->len = c->len - offset;
    out->off = c->off + offset;
    return 0;
  }
  const blk_t *b = c->b;
  uint32_t nl;
  switch (b->ref) {
  case 1: nl = b->n - offset; break;
  case 2: case 8:
    if (offset > b->n) return YO_ERR_REFERENCE_PANIC;
    nl = b->n - offset;
    break;
  case 4: {
    uint32_t bo;
    TRY(str_split16(b->cs.p, b->cs.n, offset, &bo));
    nl = str_len16(b->cs.p + bo, b->cs.n - bo);
    if (b->cs.n - bo == 1) nl = 1;
    break;
  }
  default: return YO_ERR_REFERENCE_PANIC; /* ItemContent::splice -> None .unwrap() */
  }
  out->off = offset;
  out->clock = b->clock + offset;
  out->len = nl;
  return 0;
}

typedef struct {
  VEC(car_t) cars;
  VEC(const upd_t *) ups;
} emit_t;

typedef struct {
  uint64_t c;
  uint32_t k;
  uint8_t kind;
} tiekey_t;
static int cmpk(const void *a, const void *b) {
  const tiekey_t *x = a, *y = b;
  if (x->c != y->c) return x->c < y->c ? -1 : 1;
  if (x->k != y->k) return x->k < y->k ? -1 : 1;
  return (int)x->kind - (int)y->kind;
}

#define SORT_SMALL 20 /* Rust's MAX_LEN_ALWAYS_INSERTION_SORT / MAX_INSERTION */
static int merge_blocks(upd_t *ups, size_t n, int mode, emit_t *em) {
  dec_t *decs = calloc(n + 1, sizeof(dec_t));
  dec_t **arr = malloc((n + 1) * sizeof(dec_t *));
  size_t na = 0;
  for (size_t i = 0; i < n; i++) {
    if (ups[i].clients.items == 0) continue; /* filter(!block_store.is_empty()) */
    dec_init(&decs[i], &ups[i], i);
    arr[na++] = &decs[i];
  }
  /* Sort policy per iteration (update.rs:570-590): more than SORT_SMALL live decoders ->
   * stable sort under key_less; otherwise Rust's insertion_sort_shift_left with yrs'
   * comparator.  Mode 1 runs the first regime as a binary heap keyed (client desc, clock
   * asc, last re-insert desc, input index asc) — the order a stable sort of the deque
   * keeps — and the second one as a heap too when no Item/GC tie exists (the comparator
   * is then consistent and both regimes give the heap order).  With a tie it switches to
   * the literal loop once <= SORT_SMALL decoders are live, rebuilding the deque as
   * [decoder popped last] + the rest in heap order. */
  bool use_heap = false, anomaly = false;
  dec_t *last = NULL;
  if (mode == 1) {
    size_t tot = 0;
    for (size_t i = 0; i < na; i++) tot += arr[i]->n + 1;
    tiekey_t *ks = malloc((tot + 1) * sizeof(tiekey_t));
    size_t m = 0;
    for (size_t i = 0; i < na; i++) {
      if (arr[i]->has) {
        ks[m].c = arr[i]->cur.client;
        ks[m].k = arr[i]->cur.clock;
        ks[m++].kind = arr[i]->cur.kind;
      }
      for (size_t p = arr[i]->pos; p < arr[i]->n; p++) {
        const blk_t *b = &arr[i]->u->blocks.d[arr[i]->stream[p]];
        ks[m].c = b->client;
        ks[m].k = b->clock;
        ks[m++].kind = b->kind;
      }
    }
    qsort(ks, m, sizeof(tiekey_t), cmpk);
    for (size_t i = 1; i < m; i++)
      if (ks[i].c == ks[i - 1].c && ks[i].k == ks[i - 1].k && ks[i].kind != ks[i - 1].kind) anomaly = true;
    free(ks);
    use_heap = !anomaly || na > SORT_SMALL;
  }
  dec_t **heap = NULL;
  size_t nh = 0;
  if (use_heap) {
    heap = malloc((na + 1) * sizeof(dec_t *));
    for (size_t i = 0; i < na; i++)
      if (arr[i]->has) heap_push(heap, &nh, arr[i]);
  }
  car_t cw;
  bool has_cw = false;
  int err = 0;
  int64_t iter = 0;
#define EMIT(c, up)                                                                                \
  do {                                                                                             \
    VPUSH(em->cars, c);                                                                            \
    VPUSH(em->ups, up);                                                                            \
  } while (0)
  const upd_t *cw_u = NULL;
  for (;; iter++) {
    dec_t *d;
    if (use_heap && anomaly && nh <= SORT_SMALL) { /* hand over to the literal loop */
      na = 0;
      if (last && last->has) arr[na++] = last;
      while (nh) {
        dec_t *x = heap_pop(heap, &nh);
        if (x != last) arr[na++] = x;
      }
      use_heap = false;
    }
    if (use_heap) {
      if (nh == 0) break;
      d = heap_pop(heap, &nh);
    } else {
      size_t k = 0;
      for (size_t i = 0; i < na; i++)
        if (arr[i]->has) arr[k++] = arr[i];
      na = k;
      /* Rust sort_by: insertion_sort_shift_left for len <= 20; above, the policy order */
      bool small = na <= SORT_SMALL;
      for (size_t i = 1; i < na; i++) {
        dec_t *tmp = arr[i];
        size_t j = i;
        while (j > 0 && (small ? dec_less(tmp, arr[j - 1]) : key_less(tmp, arr[j - 1]))) {
          arr[j] = arr[j - 1];
          j--;
        }
        arr[j] = tmp;
      }
      if (na == 0) break;
      d = arr[0];
    }
    last = d;
    uint64_t first_client = d->cur.client;
    if (has_cw) {
      bool iterated = false;
      uint32_t cwl = cw.clock + cw.len;
      while (d->has && (uint32_t)(d->cur.clock + d->cur.len) <= cwl && d->cur.client >= cw.client) {
        dec_next(d);
        iterated = true;
      }
      if (!d->has) goto next;
      car_t *b = &d->cur;
      if (b->client != first_client || (iterated && b->clock > cwl)) goto next;
      if (first_client != cw.client) {
        EMIT(cw, cw_u);
        cw = d->cur;
        cw_u = d->u;
        dec_next(d);
      } else if (cwl < b->clock) {
        if (cw.kind == BK_SKIP) {
          cw.len = b->clock + b->len - cw.clock;
        } else {
          EMIT(cw, cw_u);
          car_t sk = {NULL, 0, first_client, cwl, b->clock - cwl, BK_SKIP};
          cw = sk;
          cw_u = NULL;
        }
      } else {
        uint32_t diff = cwl > b->clock ? cwl - b->clock : 0;
        car_t slice;
        bool has_slice = false;
        if (diff > 0) {
          if (cw.kind == BK_SKIP)
            cw.len -= diff;
          else {
            err = car_splice(b, diff, &slice);
            if (err) goto done;
            has_slice = true;
          }
        }
        const car_t *cur = has_slice ? &slice : &d->cur;
        bool squashed = false;
        if (cw.kind == BK_SKIP && cur->kind == BK_SKIP) { /* BlockRange::merge */
          cw.len += cur->len;
          squashed = true;
        }
        if (!squashed) {
          EMIT(cw, cw_u);
          cw = has_slice ? slice : d->cur;
          cw_u = d->u;
          dec_next(d);
        }
      }
    } else {
      cw = d->cur;
      cw_u = d->u;
      has_cw = true;
      dec_next(d);
    }
    while (d->has) {
      if (d->cur.client == first_client && d->cur.clock == (uint32_t)(cw.clock + cw.len)) {
        EMIT(cw, cw_u);
        cw = d->cur;
        cw_u = d->u;
        dec_next(d);
      } else
        break;
    }
  next:
    if (use_heap && d->has) {
      d->t = iter;
      heap_push(heap, &nh, d);
    }
  }
  if (has_cw) EMIT(cw, cw_u);
done:
#undef EMIT
  for (size_t i = 0; i < n; i++) free(decs[i].stream);
  free(decs);
  free(arr);
  free(heap);
  return err;
}

/* group emitted carriers per client (UpdateBlocks::add_block) */
static size_t group_clients(const emit_t *em, clist_t **out) {
  clist_t *cl = NULL;
  size_t ncl = 0, cap = 0;
  for (size_t i = 0; i < em->cars.n; i++) {
    uint64_t c = em->cars.d[i].client;
    size_t j = 0;
    for (; j < ncl; j++)
      if (cl[j].client == c) break;
    if (j == ncl) {
      if (ncl == cap) {
        cap = cap ? cap * 2 : 8;
        cl = realloc(cl, cap * sizeof(clist_t));
      }
      memset(&cl[ncl], 0, sizeof(clist_t));
      cl[ncl].client = c;
      ncl++;
    }
    VPUSH(cl[j].cars, em->cars.d[i]);
    VPUSH(cl[j].ups, em->ups.d[i]);
  }
  *out = cl;
  return ncl;
}
static void free_clients(clist_t *cl, size_t n) {
  for (size_t i = 0; i < n; i++) {
    VFREE(cl[i].cars);
    VFREE(cl[i].ups);
  }
  free(cl);
}

/* DeleteSet merge of all inputs (update.rs:542-548, id_set.rs:385-394) */
static void merge_ds(upd_t *ups, size_t n, int mode, hb_t *res, idrvec_t *vals) {
  bool inverted = false;
  for (size_t i = 0; i < n && !inverted; i++)
    for (size_t k = 0; k < ups[i].dsv.n; k++) {
      idr_t *g = &ups[i].dsv.d[k];
      if (g->cont && g->c.e < g->c.s) inverted = true;
      for (size_t q = 0; q < g->v.n; q++)
        if (g->v.d[q].e < g->v.d[q].s) inverted = true;
    }
  bool literal = mode == 0 || inverted;
  memset(res, 0, sizeof(*res));
  for (size_t i = 0; i < n; i++) {
    upd_t *u = &ups[i];
    int32_t *ord = malloc((u->ds.items + 1) * sizeof(int32_t));
    size_t k = hb_order(&u->ds, ord);
    for (size_t q = 0; q < k; q++) {
      uint64_t client = u->ds.keys.d[ord[q]];
      const idr_t *g = &u->dsv.d[ord[q]];
      int32_t e = hb_find(res, client);
      if (e >= 0) {
        idr_merge(&vals->d[e], g);
      } else {
        bool ex;
        hb_insert(res, client, &ex);
        idr_t c;
        idr_clone(&c, g);
        VPUSH(*vals, c);
      }
    }
    free(ord);
    if (literal)
      for (size_t q = 0; q < vals->n; q++) idr_squash(&vals->d[q]);
  }
  if (!literal)
    for (size_t q = 0; q < vals->n; q++) idr_squash(&vals->d[q]);
}

/* ------------------------------------------------------------------ public API */
static int finish(wb_t *w, uint8_t **out, size_t *out_len) {
  *out = w->d ? w->d : malloc(1);
  *out_len = w->n;
  return 0;
}

int yo_merge_updates_v1(const uint8_t *const *updates, const size_t *lens, size_t n, int mode,
                        uint8_t **out, size_t *out_len) {
  *out = NULL;
  *out_len = 0;
  upd_t *ups = calloc(n + 1, sizeof(upd_t));
  int err = 0;
  bool unsupported = false;
  size_t decoded = 0;
  for (size_t i = 0; i < n; i++) {
    err = decode_update(&ups[i], updates[i], lens[i]);
    decoded = i + 1;
    if (err) break;
    if (ups[i].unsupported) unsupported = true;
  }
  wb_t w = {0};
  if (!err && unsupported) err = YO_ERR_UNSUPPORTED;
  if (!err) {
    emit_t em = {0};
    err = merge_blocks(ups, n, mode, &em);
    if (!err) {
      clist_t *cl;
      size_t ncl = group_clients(&em, &cl);
      err = encode_blocks(&w, cl, ncl, NULL);
      free_clients(cl, ncl);
    }
    VFREE(em.cars);
    VFREE(em.ups);
    if (!err) {
      hb_t res;
      idrvec_t vals = {0};
      merge_ds(ups, n, mode, &res, &vals);
      ds_encode(&w, &res, vals.d);
      for (size_t q = 0; q < vals.n; q++) idr_free(&vals.d[q]);
      VFREE(vals);
      hb_free(&res);
    }
  }
  for (size_t i = 0; i < decoded; i++) upd_free(&ups[i]);
  free(ups);
  if (err) {
    free(w.d);
    return err;
  }
  return finish(&w, out, out_len);
}

/* StateVector::decode (state_vector.rs:107-120) */
static int sv_decode_r(sv_t *sv, rd_t *rr);
static int sv_decode(sv_t *sv, const uint8_t *p, size_t n) {
  rd_t r = {p, n, 0};
  return sv_decode_r(sv, &r);
}
static int sv_decode_r(sv_t *sv, rd_t *rp) {
  memset(sv, 0, sizeof(*sv));
  rd_t r = *rp;
  uint32_t len;
  TRY(rd_var_u32(&r, &len));
  if (len && cap_to_buckets(len) * 17ull > ALLOC_LIMIT) return YO_ERR_REFERENCE_PANIC;
  hb_with_capacity(&sv->t, len);
  for (uint32_t i = 0; i < len; i++) {
    uint64_t c;
    uint32_t k;
    TRY(rd_var_u64(&r, &c));
    TRY(rd_var_u32(&r, &k));
    bool ex;
    int32_t e = hb_insert(&sv->t, c, &ex);
    if (ex)
      sv->clocks.d[e] = k;
    else
      VPUSH(sv->clocks, k);
  }
  return 0;
}
static void sv_free(sv_t *sv) {
  hb_free(&sv->t);
  VFREE(sv->clocks);
}

/* client lists of a decoded update, in stored order, Skips included */
static size_t update_clients(const upd_t *u, clist_t **out) {
  size_t nk = u->clients.keys.n;
  clist_t *cl = calloc(nk + 1, sizeof(clist_t));
  for (size_t e = 0; e < nk; e++) {
    cl[e].client = u->clients.keys.d[e];
    for (size_t k = 0; k < u->lists.d[e].idx.n; k++) {
      car_t c = car_of(&u->blocks.d[u->lists.d[e].idx.d[k]]);
      VPUSH(cl[e].cars, c);
      VPUSH(cl[e].ups, u);
    }
  }
  *out = cl;
  return nk;
}

int yo_diff_updates_v1(const uint8_t *update, size_t update_len, const uint8_t *svb, size_t sv_len,
                       uint8_t **out, size_t *out_len) {
  *out = NULL;
  *out_len = 0;
  sv_t sv;
  int err = sv_decode(&sv, svb, sv_len);
  if (err) {
    sv_free(&sv);
    return err;
  }
  upd_t u;
  err = decode_update(&u, update, update_len);
  if (!err && u.unsupported) err = YO_ERR_UNSUPPORTED;
  wb_t w = {0};
  if (!err) {
    clist_t *cl;
    size_t ncl = update_clients(&u, &cl);
    err = encode_blocks(&w, cl, ncl, &sv);
    free_clients(cl, ncl);
    if (!err) ds_encode(&w, &u.ds, u.dsv.d);
  }
  upd_free(&u);
  sv_free(&sv);
  if (err) {
    free(w.d);
    return err;
  }
  return finish(&w, out, out_len);
}

int yo_encode_state_vector_from_update_v1(const uint8_t *update, size_t len, uint8_t **out,
                                          size_t *out_len) {
  *out = NULL;
  *out_len = 0;
  upd_t u;
  int err = decode_update(&u, update, len);
  wb_t w = {0};
  if (!err) {
    /* Update::state_vector (update.rs:107-114): iterate the decoded clients table,
     * set_max into a fresh StateVector table */
    hb_t b = {0};
    VEC(uint32_t) clocks = {0};
    int32_t *ord = malloc((u.clients.items + 1) * sizeof(int32_t));
    size_t k = hb_order(&u.clients, ord);
    for (size_t i = 0; i < k && !err; i++) {
      blist_t *bl = &u.lists.d[ord[i]];
      if (bl->idx.n == 0) {
        err = YO_ERR_REFERENCE_PANIC; /* blocks[blocks.len() - 1] on an empty deque */
        break;
      }
      const blk_t *last = &u.blocks.d[bl->idx.d[bl->idx.n - 1]];
      uint32_t last_clock = last->kind == BK_ITEM ? last->clock + last->len - 1 : last->clock + last->len;
      uint32_t v = last_clock + 1;
      bool ex;
      int32_t e = hb_entry(&b, u.clients.keys.d[ord[i]], &ex);
      if (!ex) VPUSH(clocks, 0);
      if (v > clocks.d[e]) clocks.d[e] = v;
    }
    free(ord);
    if (!err) {
      wb_var(&w, b.items);
      int32_t *o2 = malloc((b.items + 1) * sizeof(int32_t));
      size_t k2 = hb_order(&b, o2);
      for (size_t i = 0; i < k2; i++) {
        wb_var(&w, b.keys.d[o2[i]]);
        wb_var(&w, clocks.d[o2[i]]);
      }
      free(o2);
    }
    hb_free(&b);
    VFREE(clocks);
  }
  upd_free(&u);
  if (err) {
    free(w.d);
    return err;
  }
  return finish(&w, out, out_len);
}

void yo_free(void *p) { free(p); }

#include "yrs_oracle_v2.c"
#include "yrs_oracle_store.c"

/* ------------------------------------------------------------------ y-sync framing
 * Message::encode / SyncMessage::encode (yrs/src/sync/protocol.rs:219-233, 245-258):
 * [MSG_SYNC = 0, step tag, varbuf(payload)]; Message::decode + SyncMessage::decode
 * (protocol.rs:179-203, 259-272) for the client's message, tags read as read_var::<u8>
 * (varint.rs:92-106).  Only SyncStep1 requests are answered: other messages are not
 * update-algebra work (UNSUPPORTED). */
static int sync_frame(uint8_t tag, uint8_t *payload, size_t n, uint8_t **out, size_t *out_len) {
  wb_t w = {0};
  wb_u8(&w, 0);
  wb_u8(&w, tag);
  wb_var(&w, n);
  wb_bytes(&w, payload, n);
  yo_free(payload);
  return finish(&w, out, out_len);
}
int yo_sync_step1_v1(const uint8_t *update, size_t len, uint8_t **out, size_t *out_len) {
  uint8_t *sv;
  size_t n;
  TRY(yo_encode_state_vector_from_update_v1(update, len, &sv, &n));
  return sync_frame(0, sv, n, out, out_len);
}
int yo_sync_step2_v1(const uint8_t *update, size_t len, const uint8_t *msg, size_t mlen, uint8_t **out,
                     size_t *out_len) {
  rd_t r = {msg, mlen, 0};
  uint32_t tag, sub;
  const uint8_t *sv;
  uint32_t svn;
  TRY(rd_var_u32(&r, &tag));
  if (tag > 255) return YO_ERR_VAR_INT;
  if (tag != 0) return YO_ERR_UNSUPPORTED;
  TRY(rd_var_u32(&r, &sub));
  if (sub > 255) return YO_ERR_VAR_INT;
  if (sub == 1 || sub == 2) return YO_ERR_UNSUPPORTED;
  if (sub != 0) return YO_ERR_UNEXPECTED_VALUE;
  TRY(rd_buf(&r, &sv, &svn));
  uint8_t *d;
  size_t n;
  TRY(yo_diff_updates_v1(update, len, sv, svn, &d, &n));
  return sync_frame(1, d, n, out, out_len);
}

/* ------------------------------------------------------------------ batch + threads (CPU baseline) */
typedef struct {
  const uint8_t *bytes, *svbytes;
  const uint64_t *upd_off, *doc_upd, *sv_off;
  size_t n_docs;
  int mode, is_diff;
  uint8_t **outs;
  size_t *lens;
  uint8_t *status;
  size_t next;
  pthread_mutex_t mu;
} job_t;

static void *worker(void *arg) {
  job_t *j = arg;
  const uint8_t **ptrs = NULL;
  size_t *lens = NULL, cap = 0;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t d0 = j->next;
    j->next += 4;
    pthread_mutex_unlock(&j->mu);
    if (d0 >= j->n_docs) break;
    for (size_t d = d0; d < d0 + 4 && d < j->n_docs; d++) {
      int st;
      const bool v2 = j->mode & 4; /* lib0 v2 batch */
      if (j->is_diff == 2) {
        st = (v2 ? yo_encode_state_vector_from_update_v2 : yo_encode_state_vector_from_update_v1)(
            j->bytes + j->upd_off[d], j->upd_off[d + 1] - j->upd_off[d], &j->outs[d], &j->lens[d]);
      } else if (j->is_diff) {
        st = (v2 ? yo_diff_updates_v2 : yo_diff_updates_v1)(j->bytes + j->upd_off[d], j->upd_off[d + 1] - j->upd_off[d],
                                                            j->svbytes + j->sv_off[d], j->sv_off[d + 1] - j->sv_off[d],
                                                            &j->outs[d], &j->lens[d]);
      } else {
        size_t u0 = j->doc_upd[d], u1 = j->doc_upd[d + 1];
        if (u1 - u0 > cap) {
          cap = u1 - u0;
          ptrs = realloc(ptrs, cap * sizeof(*ptrs));
          lens = realloc(lens, cap * sizeof(*lens));
        }
        for (size_t u = u0; u < u1; u++) {
          ptrs[u - u0] = j->bytes + j->upd_off[u];
          lens[u - u0] = j->upd_off[u + 1] - j->upd_off[u];
        }
        if (j->mode & 8) /* store-based compaction (yrs_oracle_store.c) */
          st = yo_compact_updates_v1(ptrs, lens, u1 - u0, &j->outs[d], &j->lens[d]);
        else
          st = (v2 ? yo_merge_updates_v2 : yo_merge_updates_v1)(ptrs, lens, u1 - u0, j->mode & 3, &j->outs[d],
                                                                &j->lens[d]);
      }
      j->status[d] = (uint8_t)st;
    }
  }
  free(ptrs);
  free(lens);
  return NULL;
}

static int run_batch(job_t *j, int threads, uint8_t **out, uint64_t *out_off) {
  j->outs = calloc(j->n_docs + 1, sizeof(uint8_t *));
  j->lens = calloc(j->n_docs + 1, sizeof(size_t));
  pthread_mutex_init(&j->mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t *th = malloc(threads * sizeof(pthread_t));
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, j);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&j->mu);
  uint64_t tot = 0;
  for (size_t d = 0; d < j->n_docs; d++) {
    out_off[d] = tot;
    if (j->status[d] == 0) tot += j->lens[d];
  }
  out_off[j->n_docs] = tot;
  *out = malloc(tot + 1);
  for (size_t d = 0; d < j->n_docs; d++) {
    if (j->status[d] == 0 && j->lens[d]) memcpy(*out + out_off[d], j->outs[d], j->lens[d]);
    free(j->outs[d]);
  }
  free(j->outs);
  free(j->lens);
  return 0;
}

int yo_merge_batch(const uint8_t *bytes, const uint64_t *upd_off, const uint64_t *doc_upd, size_t n_docs,
                   int mode, int threads, uint8_t **out, uint64_t *out_off, uint8_t *status) {
  job_t j;
  memset(&j, 0, sizeof(j));
  j.bytes = bytes;
  j.upd_off = upd_off;
  j.doc_upd = doc_upd;
  j.n_docs = n_docs;
  j.mode = mode;
  j.status = status;
  return run_batch(&j, threads, out, out_off);
}

int yo_diff_batch2(const uint8_t *ubytes, const uint64_t *u_off, const uint8_t *svbytes, const uint64_t *sv_off,
                   size_t n_docs, int version, int threads, uint8_t **out, uint64_t *out_off, uint8_t *status);
int yo_diff_batch(const uint8_t *ubytes, const uint64_t *u_off, const uint8_t *svbytes, const uint64_t *sv_off,
                  size_t n_docs, int threads, uint8_t **out, uint64_t *out_off, uint8_t *status) {
  return yo_diff_batch2(ubytes, u_off, svbytes, sv_off, n_docs, 1, threads, out, out_off, status);
}
/* version 1 or 2 (lib0 v2: batch mode bit 4) */
int yo_diff_batch2(const uint8_t *ubytes, const uint64_t *u_off, const uint8_t *svbytes, const uint64_t *sv_off,
                   size_t n_docs, int version, int threads, uint8_t **out, uint64_t *out_off, uint8_t *status) {
  job_t j;
  memset(&j, 0, sizeof(j));
  j.mode = version == 2 ? 4 : 0;
  j.bytes = ubytes;
  j.upd_off = u_off;
  j.svbytes = svbytes;
  j.sv_off = sv_off;
  j.n_docs = n_docs;
  j.is_diff = 1;
  j.status = status;
  return run_batch(&j, threads, out, out_off);
}

int yo_sv_batch2(const uint8_t *ubytes, const uint64_t *u_off, size_t n_docs, int version, int threads,
                 uint8_t **out, uint64_t *out_off, uint8_t *status);
int yo_sv_batch(const uint8_t *ubytes, const uint64_t *u_off, size_t n_docs, int threads, uint8_t **out,
                uint64_t *out_off, uint8_t *status) {
  return yo_sv_batch2(ubytes, u_off, n_docs, 1, threads, out, out_off, status);
}
int yo_sv_batch2(const uint8_t *ubytes, const uint64_t *u_off, size_t n_docs, int version, int threads,
                 uint8_t **out, uint64_t *out_off, uint8_t *status) {
  job_t j;
  memset(&j, 0, sizeof(j));
  j.mode = version == 2 ? 4 : 0;
  j.bytes = ubytes;
  j.upd_off = u_off;
  j.n_docs = n_docs;
  j.is_diff = 2;
  j.status = status;
  return run_batch(&j, threads, out, out_off);
}

/* StateVector decode -> encode round trip (state_vector.rs:107-130); pins the
 * hashbrown emulation against compatibility_tests.rs:293-318 */
int yo_sv_roundtrip(const uint8_t *p, size_t n, uint8_t **out, size_t *out_len) {
  sv_t sv;
  *out = NULL;
  *out_len = 0;
  int err = sv_decode(&sv, p, n);
  wb_t w = {0};
  if (!err) {
    wb_var(&w, sv.t.items);
    int32_t *o = malloc((sv.t.items + 1) * sizeof(int32_t));
    size_t k = hb_order(&sv.t, o);
    for (size_t i = 0; i < k; i++) {
      wb_var(&w, sv.t.keys.d[o[i]]);
      wb_var(&w, sv.clocks.d[o[i]]);
    }
    free(o);
  }
  sv_free(&sv);
  if (err) {
    free(w.d);
    return err;
  }
  return finish(&w, out, out_len);
}

/* byte offset where the DeleteSet starts (test helper for order-insensitive checks) */
int yo_ds_offset(const uint8_t *p, size_t n, size_t *off) {
  upd_t u;
  memset(&u, 0, sizeof(u));
  u.base = p;
  u.len = n;
  rd_t r = {p, n, 0};
  uint32_t ncl;
  int err = rd_var_u32(&r, &ncl);
  for (uint32_t i = 0; i < ncl && !err; i++) {
    uint32_t nb, c32, clock;
    if ((err = rd_var_u32(&r, &nb)) || (err = rd_var_u32(&r, &c32)) || (err = rd_var_u32(&r, &clock))) break;
    for (uint32_t j = 0; j < nb && !err; j++) {
      blk_t b;
      bool has;
      err = decode_block(&u, &r, c32, clock, &b, &has);
      if (!err && has) clock += b.len;
    }
  }
  *off = r.i;
  VFREE(u.elems);
  return err;
}
