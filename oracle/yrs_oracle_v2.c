/*
 * yrs_oracle_v2.c — TEST INFRASTRUCTURE ONLY (included by yrs_oracle.c).
 *
 * lib0 v2 restatement: merge_updates_v2 / diff_updates_v2 /
 * encode_state_vector_from_update_v2 (yrs/src/alt.rs:35-48, 63-66, 88-97).  The decoded
 * model, the merge loop, the DeleteSet merge and the hash-table orders are the v1 ones;
 * only the primitives differ:
 *   DecoderV2        yrs/src/updates/decoder.rs:193-370 (feature flag, 9 column buffers,
 *                    rest cursor; read_usize panics instead of failing past 64 bits or
 *                    past the end of the buffer)
 *   IntDiffOptRle    decoder.rs:372-405     UIntOptRle decoder.rs:407-438
 *   Rle              decoder.rs:440-467     StringDecoder decoder.rs:469-504 (UTF-16 counts)
 *   key cache        decoder.rs:355-364 / encoder.rs write_key (key_table never updated)
 *   EncoderV2        yrs/src/updates/encoder.rs:182-528 (column encoders, to_vec layout)
 *   DeleteSet        read_ds_clock/len, write_ds_clock/len (diff-coded, len - 1)
 * Policies (as for v1): an arithmetic overflow that debug Rust panics on, an out-of-range
 * index or a str slice off a char boundary -> REFERENCE_PANIC.  Embed/Format values are
 * Any bytes in v2 (read_json = Any::decode), kept as spans (blk_t.json_any) and re-encoded
 * canonically.
 */

/* ------------------------------------------------------------------ column decoders */
typedef struct {
  rd_t c;
  uint32_t last, count;
  int32_t diff;
} icol_t; /* IntDiffOptRleDecoder */
typedef struct {
  rd_t c;
  uint64_t last;
  uint32_t count;
} ucol_t; /* UIntOptRleDecoder */
typedef struct {
  rd_t c;
  uint8_t last;
  int32_t count;
} rcol_t; /* RleDecoder */
typedef struct {
  const uint8_t *s;
  size_t n, pos;
  ucol_t lens;
} scol_t; /* StringDecoder */

/* SignedVarInt::read_signed for i64 (varint.rs): magnitude + sign (-0 is negative) */
static int rd_var_signed(rd_t *r, uint64_t *mag, bool *neg) {
  uint8_t b;
  TRY(rd_u8(r, &b));
  uint64_t num = b & 0x3f;
  unsigned len = 6;
  *neg = (b & 0x40) != 0;
  if (b & 0x80) {
    for (;;) {
      TRY(rd_u8(r, &b));
      num |= (uint64_t)(b & 0x7f) << (len & 63);
      len += 7;
      if (b < 0x80) break;
      if (len > 70) return YO_ERR_VAR_INT;
    }
  }
  *mag = num;
  return 0;
}

static int icol_read(icol_t *d, uint32_t *v) {
  if (d->count == 0) {
    int64_t x;
    TRY(rd_var_i64(&d->c, &x)); /* read_var::<i32>: i64 then try_into */
    if (x < INT32_MIN || x > INT32_MAX) return YO_ERR_VAR_INT;
    const int32_t diff = (int32_t)x;
    d->diff = diff >> 1;
    if (diff & 1) {
      uint32_t c;
      TRY(rd_var_u32(&d->c, &c));
      if (c > UINT32_MAX - 2) return YO_ERR_REFERENCE_PANIC; /* u32 + 2 overflow */
      d->count = c + 2;
    } else {
      d->count = 1;
    }
  }
  const int64_t nv = (int64_t)(int32_t)d->last + d->diff;
  if (nv < INT32_MIN || nv > INT32_MAX) return YO_ERR_REFERENCE_PANIC; /* i32 add overflow */
  d->last = (uint32_t)(int32_t)nv;
  d->count--;
  *v = d->last;
  return 0;
}
static int ucol_read(ucol_t *d, uint64_t *v) {
  if (d->count == 0) {
    uint64_t mag;
    bool neg;
    TRY(rd_var_signed(&d->c, &mag, &neg));
    if (neg) {
      uint32_t c;
      TRY(rd_var_u32(&d->c, &c));
      if (c > UINT32_MAX - 2) return YO_ERR_REFERENCE_PANIC;
      d->count = c + 2;
    } else {
      d->count = 1;
    }
    d->last = mag; /* (-s.value()) as u64 for negatives, s.value() as u64 otherwise */
  }
  d->count--;
  *v = d->last;
  return 0;
}
static int rcol_read(rcol_t *d, uint8_t *v) {
  if (d->count == 0) {
    TRY(rd_u8(&d->c, &d->last));
    if (d->c.i < d->c.n) {
      uint32_t c;
      TRY(rd_var_u32(&d->c, &c));
      if ((int32_t)c == INT32_MAX) return YO_ERR_REFERENCE_PANIC; /* (c as i32) + 1 overflow */
      d->count = (int32_t)c + 1;
    } else {
      d->count = -1; /* read the current value forever */
    }
  }
  d->count--;
  *v = d->last;
  return 0;
}
/* StringDecoder::read_str: `remaining` UTF-16 units, chars() over the column (unchecked
 * UTF-8, decoded like core's next_code_point); usize underflow and a slice end off a char
 * boundary panic */
static int scol_read(scol_t *d, span_t *out) {
  uint64_t remaining;
  TRY(ucol_read(&d->lens, &remaining));
  size_t i = 0, j = d->pos;
  while (j < d->n) {
    if (remaining == 0) break;
    const uint32_t c = utf8_next(d->s, d->n, &j);
    i += ch_len8(c);
    const uint32_t u = ch_len16(c);
    if (remaining < u) return YO_ERR_REFERENCE_PANIC;
    remaining -= u;
  }
  const size_t len = d->n - d->pos;
  if (i > len || (i < len && (int8_t)d->s[d->pos + i] < -0x40)) return YO_ERR_REFERENCE_PANIC;
  out->p = d->s + d->pos;
  out->n = (uint32_t)i;
  d->pos += i;
  return 0;
}

/* DecoderV2::read_usize + read_buf (decoder.rs:246-277) */
static int usize_buf(const uint8_t *p, size_t n, size_t *idx, span_t *out) {
  if (*idx >= n) return YO_ERR_VAR_INT;
  uint64_t num = 0;
  unsigned len = 0;
  for (;;) {
    if (*idx >= n) return YO_ERR_REFERENCE_PANIC; /* buf[*idx] out of bounds */
    const uint8_t b = p[(*idx)++];
    if (len >= 64) return YO_ERR_REFERENCE_PANIC; /* usize shift overflow */
    num |= (uint64_t)(b & 127) << len;
    len += 7;
    if (b < 128) break;
    if (len > 128) return YO_ERR_VAR_INT;
  }
  /* start + len overflows usize (decoder.rs:268-269): a debug build panics on the add, a
   * release build on &buf[start..end] with the wrapped end below start */
  if (num > UINT64_MAX - (uint64_t)*idx) return YO_ERR_REFERENCE_PANIC;
  if (num > n - *idx) return YO_ERR_EOS;
  out->p = p + *idx;
  out->n = (uint32_t)num;
  *idx += (size_t)num;
  return 0;
}

typedef struct {
  rd_t r; /* rest cursor */
  icol_t keyc, lclk, rclk;
  ucol_t cli, tref, len;
  rcol_t info, pinfo;
  scol_t str;
  VEC(span_t) keys;
  uint32_t ds_cur;
} dec2_t;

static rd_t rd_of(span_t s) {
  rd_t r = {s.p, s.n, 0};
  return r;
}
/* DecoderV2::new (decoder.rs:209-244) */
static int dec2_init(dec2_t *d, const uint8_t *p, size_t n) {
  memset(d, 0, sizeof(*d));
  size_t idx = n > 0 ? 1 : 0; /* feature flag */
  span_t col[9];
  for (int k = 0; k < 9; k++) TRY(usize_buf(p, n, &idx, &col[k]));
  d->r.p = p + idx;
  d->r.n = n - idx;
  d->r.i = 0;
  d->keyc.c = rd_of(col[0]);
  d->cli.c = rd_of(col[1]);
  d->lclk.c = rd_of(col[2]);
  d->rclk.c = rd_of(col[3]);
  d->info.c = rd_of(col[4]);
  d->pinfo.c = rd_of(col[6]);
  d->tref.c = rd_of(col[7]);
  d->len.c = rd_of(col[8]);
  /* StringDecoder::new: the column is [usize len][string bytes][UIntOptRle lengths] */
  size_t si = 0;
  span_t sb;
  TRY(usize_buf(col[5].p, col[5].n, &si, &sb));
  d->str.s = sb.p;
  d->str.n = sb.n;
  d->str.pos = 0;
  d->str.lens.c = (rd_t){col[5].p, col[5].n, si};
  return 0;
}
static void dec2_free(dec2_t *d) { VFREE(d->keys); }

static int d2_len(dec2_t *d, uint32_t *v) {
  uint64_t x;
  TRY(ucol_read(&d->len, &x));
  *v = (uint32_t)x; /* read_len: u64 as u32 */
  return 0;
}
static int d2_key(dec2_t *d, span_t *out) {
  uint32_t kc;
  TRY(icol_read(&d->keyc, &kc));
  if (kc < d->keys.n) {
    *out = d->keys.d[kc];
    return 0;
  }
  TRY(scol_read(&d->str, out));
  VPUSH(d->keys, *out);
  return 0;
}
/* read_ds_clock / read_ds_len (decoder.rs:302-311) */
static int d2_ds_clock(dec2_t *d, uint32_t *v) {
  uint32_t x;
  TRY(rd_var_u32(&d->r, &x));
  if ((uint64_t)d->ds_cur + x > UINT32_MAX) return YO_ERR_REFERENCE_PANIC;
  d->ds_cur += x;
  *v = d->ds_cur;
  return 0;
}
static int d2_ds_len(dec2_t *d, uint32_t *v) {
  uint32_t x;
  TRY(rd_var_u32(&d->r, &x));
  if (x == UINT32_MAX) return YO_ERR_REFERENCE_PANIC;
  const uint32_t diff = x + 1;
  if ((uint64_t)d->ds_cur + diff > UINT32_MAX) return YO_ERR_REFERENCE_PANIC;
  d->ds_cur += diff;
  *v = diff;
  return 0;
}

/* ItemContent::decode (block.rs:1786-1835) over DecoderV2 */
static int content_decode2(upd_t *u, dec2_t *d, uint8_t ref, blk_t *b) {
  rd_t *r = &d->r;
  uint32_t n32;
  switch (ref) {
  case 1: TRY(d2_len(d, &b->n)); b->len = b->n; return 0;
  case 2: {
    TRY(d2_len(d, &n32));
    int32_t remaining = (int32_t)n32;
    if (remaining < 0) return YO_ERR_NOT_ENOUGH_MEMORY;
    b->e0 = (uint32_t)u->elems.n;
    b->n = 0;
    while (remaining >= 0) {
      span_t s;
      TRY(scol_read(&d->str, &s));
      VPUSH(u->elems, s);
      b->n++;
      remaining--;
    }
    b->len = b->n;
    return 0;
  }
  case 3: TRY(rd_buf(r, &b->cs.p, &b->cs.n)); b->len = 1; return 0;
  case 4: TRY(scol_read(&d->str, &b->cs)); b->len = str_len16(b->cs.p, b->cs.n); return 0;
  case 5: case 6: { /* read_json = Any::decode on the rest cursor */
    span_t *js = &b->cs;
    if (ref == 6) {
      TRY(d2_key(d, &b->cs));
      js = &b->cs2;
    }
    const size_t st = r->i;
    TRY(any_skip2(r, 0, true));
    js->p = r->p + st;
    js->n = (uint32_t)(r->i - st);
    b->json_any = 1;
    b->len = 1;
    return 0;
  }
  case 7: {
    uint64_t t;
    TRY(ucol_read(&d->tref, &t));
    b->tref = (uint8_t)t; /* read_type_ref: u64 as u8 */
    b->len = 1;
    switch (b->tref) {
    case 0: case 1: case 2: case 4: case 5: case 6: case 9: case 15: return 0;
    case 3: return d2_key(d, &b->cs);
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
    TRY(d2_len(d, &b->n));
    if ((uint64_t)b->n * 24 > ALLOC_LIMIT) return YO_ERR_NOT_ENOUGH_MEMORY;
    b->e0 = (uint32_t)u->elems.n;
    for (uint32_t i = 0; i < b->n; i++) {
      span_t s;
      s.p = r->p + r->i;
      const size_t st = r->i;
      TRY(any_skip2(r, 0, true));
      s.n = (uint32_t)(r->i - st);
      VPUSH(u->elems, s);
    }
    b->len = b->n;
    return 0;
  }
  case 9:
    TRY(scol_read(&d->str, &b->cs)); /* Options::decode: read_string (guid) */
    TRY(doc_options_any(u, r, b));
    b->len = 1;
    return 0;
  case 11: {
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

/* Update::decode_block (update.rs:433-488) over DecoderV2 */
static int decode_block2(upd_t *u, dec2_t *d, uint64_t client, uint32_t clock, blk_t *b, bool *has) {
  memset(b, 0, sizeof(*b));
  b->client = client;
  b->clock = clock;
  uint8_t info;
  TRY(rcol_read(&d->info, &info));
  *has = true;
  if (info == 10 || info == 0) {
    b->kind = info == 10 ? BK_SKIP : BK_GC;
    return d2_len(d, &b->len);
  }
  b->kind = BK_ITEM;
  const bool cant_copy = (info & 0xC0) == 0;
  if (info & 0x80) { /* read_left_id */
    TRY(ucol_read(&d->cli, &b->oc));
    TRY(icol_read(&d->lclk, &b->ok));
    b->has_origin = 1;
  }
  if (info & 0x40) { /* read_right_id */
    TRY(ucol_read(&d->cli, &b->rc));
    TRY(icol_read(&d->rclk, &b->rk));
    b->has_ro = 1;
  }
  if (cant_copy) {
    uint8_t pi;
    TRY(rcol_read(&d->pinfo, &pi));
    if (pi == 1) { /* read_parent_info: == 1 */
      b->pkind = PK_NAMED;
      TRY(scol_read(&d->str, &b->pname));
    } else {
      b->pkind = PK_ID;
      TRY(ucol_read(&d->cli, &b->pc));
      TRY(icol_read(&d->lclk, &b->pk));
    }
    if (info & 0x20) {
      b->has_psub = 1;
      TRY(scol_read(&d->str, &b->psub));
    }
  }
  b->ref = info & 15;
  TRY(content_decode2(u, d, b->ref, b));
  if (b->len == 0) *has = false;
  return 0;
}

/* Decode for Update (update.rs:714-749) + IdSet::decode (id_set.rs:412-426) over DecoderV2 */
static int decode_update2_body(upd_t *u, dec2_t *d) {
  rd_t *r = &d->r;
  uint32_t ncl;
  TRY(rd_var_u32(r, &ncl));
  TRY(hb_reserve(&u->clients, ncl, 40, true));
  for (uint32_t i = 0; i < ncl; i++) {
    uint32_t nb, clock;
    uint64_t client;
    TRY(rd_var_u32(r, &nb));
    TRY(ucol_read(&d->cli, &client)); /* read_client: u64 */
    TRY(rd_var_u32(r, &clock));
    bool existed;
    const int32_t e = hb_entry(&u->clients, client, &existed);
    if (!existed) {
      blist_t bl = {0};
      VPUSH(u->lists, bl);
    }
    if (((uint64_t)u->lists.d[e].idx.n + nb) * 32 > ALLOC_LIMIT) return YO_ERR_NOT_ENOUGH_MEMORY;
    for (uint32_t j = 0; j < nb; j++) {
      blk_t b;
      bool has;
      TRY(decode_block2(u, d, client, clock, &b, &has));
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
  TRY(rd_var_u32(r, &nds));
  for (uint32_t i = 0; i < nds; i++) {
    d->ds_cur = 0; /* reset_ds_cur_val */
    uint32_t c32, nr;
    TRY(rd_var_u32(r, &c32));
    TRY(rd_var_u32(r, &nr));
    idr_t g;
    memset(&g, 0, sizeof(g));
    int e = 0;
    if (nr == 1) {
      uint32_t c, l;
      e = d2_ds_clock(d, &c);
      if (!e) e = d2_ds_len(d, &l);
      if (!e) {
        g.cont = 1;
        g.c.s = c;
        g.c.e = c + l;
      }
    } else {
      for (uint32_t k = 0; k < nr && !e; k++) {
        uint32_t c, l;
        e = d2_ds_clock(d, &c);
        if (!e) e = d2_ds_len(d, &l);
        if (!e) {
          rng_t x = {c, c + l};
          VPUSH(g.v, x);
        }
      }
    }
    if (e) {
      idr_free(&g);
      return e;
    }
    bool existed;
    const int32_t k = hb_insert(&u->ds, c32, &existed);
    if (existed) {
      idr_free(&u->dsv.d[k]);
      u->dsv.d[k] = g;
    } else
      VPUSH(u->dsv, g);
  }
  return 0;
}
static int decode_update2(upd_t *u, const uint8_t *p, size_t n) {
  memset(u, 0, sizeof(*u));
  u->base = p;
  u->len = n;
  dec2_t d;
  int e = dec2_init(&d, p, n);
  if (!e) e = decode_update2_body(u, &d);
  dec2_free(&d);
  return e;
}
static int sv_decode2(sv_t *sv, const uint8_t *p, size_t n) {
  dec2_t d;
  memset(sv, 0, sizeof(*sv));
  int e = dec2_init(&d, p, n);
  if (!e) e = sv_decode_r(sv, &d.r);
  dec2_free(&d);
  return e;
}

/* ------------------------------------------------------------------ column encoders */
typedef struct {
  wb_t b;
  uint32_t last, count;
  int32_t diff;
} ienc_t; /* IntDiffOptRleEncoder */
typedef struct {
  wb_t b;
  uint64_t last;
  uint32_t count;
} uenc_t; /* UIntOptRleEncoder */
typedef struct {
  wb_t b;
  int has;
  uint8_t last;
  uint32_t count;
} renc_t; /* RleEncoder */

/* SignedVarInt::write_signed (varint.rs): sign bit from `neg`, magnitude `mag` */
static void wb_signed(wb_t *w, uint64_t mag, bool neg) {
  wb_u8(w, (uint8_t)((mag > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (uint8_t)(mag & 63)));
  mag >>= 6;
  while (mag > 0) {
    wb_u8(w, (uint8_t)((mag > 127 ? 0x80 : 0) | (uint8_t)(mag & 127)));
    mag >>= 7;
  }
}
static void ienc_flush(ienc_t *e) {
  if (e->count > 0) {
    const int32_t ed = (int32_t)((uint32_t)e->diff << 1) | (e->count == 1 ? 0 : 1);
    wb_var_i64(&e->b, ed);
    if (e->count > 1) wb_var(&e->b, e->count - 2);
  }
}
static void ienc_write(ienc_t *e, uint32_t v) {
  const int32_t diff = (int32_t)(v - e->last);
  if (e->diff == diff) {
    e->last = v;
    e->count++;
  } else {
    ienc_flush(e);
    e->count = 1;
    e->diff = diff;
    e->last = v;
  }
}
static void uenc_flush(uenc_t *e) {
  if (e->count > 0) {
    if (e->count == 1) {
      wb_var_i64(&e->b, (int64_t)e->last);
    } else {
      wb_signed(&e->b, e->last, true);
      wb_var(&e->b, e->count - 2);
    }
  }
}
static void uenc_write(uenc_t *e, uint64_t v) {
  if (e->last == v) {
    e->count++;
  } else {
    uenc_flush(e);
    e->count = 1;
    e->last = v;
  }
}
static void renc_write(renc_t *e, uint8_t v) {
  if (e->has && e->last == v) {
    e->count++;
  } else {
    if (e->count > 0) wb_var(&e->b, e->count - 1);
    e->count = 1;
    wb_u8(&e->b, v);
    e->last = v;
    e->has = 1;
  }
}
/* str.encode_utf16().count() over chars() of the (unchecked) bytes */
static uint32_t utf16_count(const uint8_t *s, uint32_t n) {
  uint32_t k = 0;
  size_t i = 0;
  while (i < n) k += ch_len16(utf8_next(s, n, &i));
  return k;
}

typedef struct {
  ienc_t keyc, lclk, rclk;
  uenc_t cli, tref, len, slen;
  renc_t info, pinfo;
  wb_t sbuf, rest;
  uint32_t seq, ds_cur;
} enc2_t;

static void e2_string(enc2_t *e, const uint8_t *p, uint32_t n) {
  wb_bytes(&e->sbuf, p, n);
  uenc_write(&e->slen, utf16_count(p, n));
}
static void e2_left_id(enc2_t *e, uint64_t client, uint32_t clock) {
  uenc_write(&e->cli, client);
  ienc_write(&e->lclk, clock);
}
static void e2_right_id(enc2_t *e, uint64_t client, uint32_t clock) {
  uenc_write(&e->cli, client);
  ienc_write(&e->rclk, clock);
}
static void e2_key(enc2_t *e, const uint8_t *p, uint32_t n) {
  ienc_write(&e->keyc, e->seq++);
  e2_string(e, p, n); /* key_table is never filled: every key is written */
}
static void e2_any(enc2_t *e, span_t s) {
  rd_t r = {s.p, s.n, 0};
  any_encode(&r, &e->rest);
}
static void e2_ds_clock(enc2_t *e, uint32_t c) {
  wb_var(&e->rest, (uint32_t)(c - e->ds_cur));
  e->ds_cur = c;
}
static void e2_ds_len(enc2_t *e, uint32_t l) {
  wb_var(&e->rest, (uint32_t)(l - 1));
  e->ds_cur += l;
}
/* EncoderV2::to_vec (encoder.rs:236-259) */
static int e2_finish(enc2_t *e, uint8_t **out, size_t *out_len) {
  ienc_flush(&e->keyc);
  uenc_flush(&e->cli);
  ienc_flush(&e->lclk);
  ienc_flush(&e->rclk);
  uenc_flush(&e->tref);
  uenc_flush(&e->len);
  uenc_flush(&e->slen);
  wb_t str = {0};
  wb_str(&str, e->sbuf.d, (uint32_t)e->sbuf.n);
  wb_bytes(&str, e->slen.b.d, e->slen.b.n);
  wb_t w = {0};
  wb_u8(&w, 0);
  const wb_t *cols[9] = {&e->keyc.b, &e->cli.b, &e->lclk.b, &e->rclk.b, &e->info.b, &str, &e->pinfo.b,
                         &e->tref.b, &e->len.b};
  for (int k = 0; k < 9; k++) wb_str(&w, cols[k]->d, (uint32_t)cols[k]->n);
  wb_bytes(&w, e->rest.d, e->rest.n);
  VFREE(str);
  wb_t *all[12] = {&e->keyc.b, &e->cli.b, &e->lclk.b, &e->rclk.b, &e->info.b, &e->pinfo.b, &e->tref.b,
                   &e->len.b, &e->slen.b, &e->sbuf, &e->rest, NULL};
  for (int k = 0; all[k]; k++) VFREE(*all[k]);
  return finish(&w, out, out_len);
}
static void e2_free(enc2_t *e) {
  wb_t *all[12] = {&e->keyc.b, &e->cli.b, &e->lclk.b, &e->rclk.b, &e->info.b, &e->pinfo.b, &e->tref.b,
                   &e->len.b, &e->slen.b, &e->sbuf, &e->rest, NULL};
  for (int k = 0; all[k]; k++) VFREE(*all[k]);
}

/* ItemSlice::encode (slice.rs:199-251) + ItemContent::encode_slice (block.rs:1711-1754) over EncoderV2 */
static int encode_item2(enc2_t *e, const upd_t *u, const blk_t *b, uint32_t off) {
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
  const bool cant_copy = (info & 0xC0) == 0;
  renc_write(&e->info, info);
  if (origin) e2_left_id(e, oc, ok);
  if (b->has_ro) e2_right_id(e, b->rc, b->rk);
  if (cant_copy) {
    if (b->pkind == PK_NAMED) {
      renc_write(&e->pinfo, 1);
      e2_string(e, b->pname.p, b->pname.n);
    } else if (b->pkind == PK_ID) {
      renc_write(&e->pinfo, 0);
      e2_left_id(e, b->pc, b->pk);
    } else
      return YO_ERR_REFERENCE_PANIC;
    if (b->has_psub) e2_string(e, b->psub.p, b->psub.n);
  }
  const uint32_t end = b->len - 1;
  switch (b->ref) {
  case 1: uenc_write(&e->len, (uint32_t)(end - off + 1)); return 0;
  case 2:
    uenc_write(&e->len, (uint32_t)(end - off + 1));
    for (uint32_t i = off; i <= end && i < b->n; i++) e2_string(e, u->elems.d[b->e0 + i].p, u->elems.d[b->e0 + i].n);
    return 0;
  case 3: wb_str(&e->rest, b->cs.p, b->cs.n); return 0;
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
    e2_string(e, s, n);
    return 0;
  }
  case 5:
  case 6:
    if (!b->json_any) return YO_ERR_UNSUPPORTED; /* v1 JSON text never reaches a v2 encoder */
    if (b->ref == 6) e2_key(e, b->cs.p, b->cs.n);
    e2_any(e, b->ref == 6 ? b->cs2 : b->cs);
    return 0;
  case 7:
    uenc_write(&e->tref, b->tref);
    if (b->tref == 3) e2_key(e, b->cs.p, b->cs.n);
    if (b->tref == 7) {
      const bool single = b->sc == b->ec && b->sk == b->ek;
      wb_u8(&e->rest, (uint8_t)((single ? 0 : 1) | (b->mflags & 2) | (b->mflags & 4)));
      wb_var(&e->rest, b->sc);
      wb_var(&e->rest, b->sk);
      if (!single) {
        wb_var(&e->rest, b->ec);
        wb_var(&e->rest, b->ek);
      }
    }
    return 0;
  case 8:
    uenc_write(&e->len, (uint32_t)(end - off + 1));
    for (uint32_t i = off; i <= end && i < b->n; i++) e2_any(e, u->elems.d[b->e0 + i]);
    return 0;
  case 9: { /* Options::encode: write_string(guid) + write_any(options) */
    e2_string(e, b->cs.p, b->cs.n);
    wb_t *w = &e->rest;
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
    wb_u8(w, b->doc_auto_load ? 120 : 121);
    return 0;
  }
  case 11: {
    const bool collapsed = b->sc == b->ec && b->sk == b->ek;
    const int32_t fl = (int32_t)b->mflags;
    const int32_t prio = fl >> 6;
    int32_t bb = (collapsed ? 1 : 0) | ((fl & 2) ? 2 : 0) | ((fl & 4) ? 4 : 0);
    bb |= (int32_t)((uint32_t)prio << 6);
    wb_var_i64(&e->rest, bb);
    wb_var(&e->rest, b->sc);
    wb_var(&e->rest, b->sk);
    if (!collapsed) {
      wb_var(&e->rest, b->ec);
      wb_var(&e->rest, b->ek);
    }
    return 0;
  }
  }
  return YO_ERR_REFERENCE_PANIC;
}
static int encode_carrier2(enc2_t *e, const upd_t *u, const car_t *c, uint32_t offset) {
  if (c->kind == BK_SKIP || c->kind == BK_GC) {
    renc_write(&e->info, c->kind == BK_SKIP ? 10 : 0);
    uenc_write(&e->len, (uint32_t)(c->len - offset));
    return 0;
  }
  return encode_item2(e, u, c->b, c->off + offset);
}
/* encode_diff (update.rs:490-535) over EncoderV2: same selection as encode_blocks */
static int encode_blocks2(enc2_t *e, clist_t *cl, size_t ncl, const sv_t *sv) {
  typedef struct {
    uint64_t client;
    uint32_t offset;
    size_t first, ci;
  } sel_t;
  sel_t *sel = malloc((ncl + 1) * sizeof(sel_t));
  size_t ns = 0;
  for (size_t i = 0; i < ncl; i++) {
    const uint32_t remote = sv_get(sv, cl[i].client);
    for (size_t k = 0; k < cl[i].cars.n; k++) {
      const car_t *c = &cl[i].cars.d[k];
      if (c->kind == BK_SKIP) continue;
      if ((uint32_t)(c->clock + c->len) > remote) {
        const int64_t o = (int64_t)remote - (int64_t)c->clock;
        sel[ns].client = cl[i].client;
        sel[ns].offset = o > 0 ? (uint32_t)o : 0;
        sel[ns].first = k;
        sel[ns].ci = i;
        ns++;
        break;
      }
    }
  }
  for (size_t i = 1; i < ns; i++) {
    sel_t t = sel[i];
    size_t j = i;
    while (j > 0 && sel[j - 1].client < t.client) {
      sel[j] = sel[j - 1];
      j--;
    }
    sel[j] = t;
  }
  wb_var(&e->rest, ns);
  for (size_t s = 0; s < ns; s++) {
    clist_t *c = &cl[sel[s].ci];
    wb_var(&e->rest, c->cars.n - sel[s].first);
    uenc_write(&e->cli, c->client); /* write_client */
    const car_t *f = &c->cars.d[sel[s].first];
    wb_var(&e->rest, (uint32_t)(f->clock + sel[s].offset));
    for (size_t k = sel[s].first; k < c->cars.n; k++) {
      const int err = encode_carrier2(e, c->ups.d[k], &c->cars.d[k], k == sel[s].first ? sel[s].offset : 0);
      if (err) {
        free(sel);
        return err;
      }
    }
  }
  free(sel);
  return 0;
}
/* IdSet::encode (id_set.rs:401-410) + IdRange::encode_raw / Range::encode over EncoderV2 */
static void idr_encode_raw2(enc2_t *e, const idr_t *r) {
  if (r->cont) {
    wb_var(&e->rest, 1);
    e2_ds_clock(e, r->c.s);
    e2_ds_len(e, (uint32_t)(r->c.e - r->c.s));
  } else {
    wb_var(&e->rest, (uint32_t)r->v.n);
    for (size_t i = 0; i < r->v.n; i++) {
      e2_ds_clock(e, r->v.d[i].s);
      e2_ds_len(e, (uint32_t)(r->v.d[i].e - r->v.d[i].s));
    }
  }
}
static void ds_encode2(enc2_t *e, const hb_t *t, const idr_t *vals) {
  wb_var(&e->rest, (uint32_t)t->items);
  int32_t *ord = malloc((t->items + 1) * sizeof(int32_t));
  const size_t k = hb_order(t, ord);
  for (size_t i = 0; i < k; i++) {
    e->ds_cur = 0; /* reset_ds_cur_val */
    wb_var(&e->rest, t->keys.d[ord[i]]);
    const idr_t *r = &vals[ord[i]];
    if (idr_is_squashed(r)) {
      idr_encode_raw2(e, r);
    } else {
      idr_t c;
      idr_clone(&c, r);
      idr_squash(&c);
      idr_encode_raw2(e, &c);
      idr_free(&c);
    }
  }
  free(ord);
}

/* ------------------------------------------------------------------ public API (alt.rs:35-48, 63-66, 88-97) */
/* in_v1: the inputs are v1 (Update::decode_v1), the merged Update still encoded with EncoderV2:
 * Update::merge_updates(us).encode_v2() -- what yconvert_updates_v1_to_v2_batch_device computes
 * per update (the DeleteSet keeps the merged map's order, no v1 round trip in between). */
static int merge_to_v2(const uint8_t *const *updates, const size_t *lens, size_t n, int mode, bool in_v1,
                       uint8_t **out, size_t *out_len) {
  *out = NULL;
  *out_len = 0;
  upd_t *ups = calloc(n + 1, sizeof(upd_t));
  int err = 0;
  bool unsupported = false;
  size_t decoded = 0;
  for (size_t i = 0; i < n; i++) {
    err = in_v1 ? decode_update(&ups[i], updates[i], lens[i]) : decode_update2(&ups[i], updates[i], lens[i]);
    decoded = i + 1;
    if (err) break;
    if (ups[i].unsupported) unsupported = true;
  }
  enc2_t e;
  memset(&e, 0, sizeof(e));
  if (!err && unsupported) err = YO_ERR_UNSUPPORTED;
  if (!err) {
    emit_t em = {0};
    err = merge_blocks(ups, n, mode, &em);
    if (!err) {
      clist_t *cl;
      const size_t ncl = group_clients(&em, &cl);
      err = encode_blocks2(&e, cl, ncl, NULL);
      free_clients(cl, ncl);
    }
    VFREE(em.cars);
    VFREE(em.ups);
    if (!err) {
      hb_t res;
      idrvec_t vals = {0};
      merge_ds(ups, n, mode, &res, &vals);
      ds_encode2(&e, &res, vals.d);
      for (size_t q = 0; q < vals.n; q++) idr_free(&vals.d[q]);
      VFREE(vals);
      hb_free(&res);
    }
  }
  for (size_t i = 0; i < decoded; i++) upd_free(&ups[i]);
  free(ups);
  if (err) {
    e2_free(&e);
    return err;
  }
  return e2_finish(&e, out, out_len);
}

int yo_merge_updates_v2(const uint8_t *const *updates, const size_t *lens, size_t n, int mode, uint8_t **out,
                        size_t *out_len) {
  return merge_to_v2(updates, lens, n, mode, false, out, out_len);
}
int yo_merge_updates_v1_to_v2(const uint8_t *const *updates, const size_t *lens, size_t n, int mode, uint8_t **out,
                              size_t *out_len) {
  return merge_to_v2(updates, lens, n, mode, true, out, out_len);
}

int yo_diff_updates_v2(const uint8_t *update, size_t update_len, const uint8_t *svb, size_t sv_len, uint8_t **out,
                       size_t *out_len) {
  *out = NULL;
  *out_len = 0;
  sv_t sv;
  int err = sv_decode2(&sv, svb, sv_len);
  if (err) {
    sv_free(&sv);
    return err;
  }
  upd_t u;
  err = decode_update2(&u, update, update_len);
  if (!err && u.unsupported) err = YO_ERR_UNSUPPORTED;
  enc2_t e;
  memset(&e, 0, sizeof(e));
  if (!err) {
    clist_t *cl;
    const size_t ncl = update_clients(&u, &cl);
    err = encode_blocks2(&e, cl, ncl, &sv);
    free_clients(cl, ncl);
    if (!err) ds_encode2(&e, &u.ds, u.dsv.d);
  }
  upd_free(&u);
  sv_free(&sv);
  if (err) {
    e2_free(&e);
    return err;
  }
  return e2_finish(&e, out, out_len);
}

int yo_encode_state_vector_from_update_v2(const uint8_t *update, size_t len, uint8_t **out, size_t *out_len) {
  *out = NULL;
  *out_len = 0;
  upd_t u;
  int err = decode_update2(&u, update, len);
  enc2_t e;
  memset(&e, 0, sizeof(e));
  if (!err) {
    hb_t b = {0};
    VEC(uint32_t) clocks = {0};
    int32_t *ord = malloc((u.clients.items + 1) * sizeof(int32_t));
    const size_t k = hb_order(&u.clients, ord);
    for (size_t i = 0; i < k && !err; i++) {
      const blist_t *bl = &u.lists.d[ord[i]];
      if (bl->idx.n == 0) {
        err = YO_ERR_REFERENCE_PANIC;
        break;
      }
      const blk_t *last = &u.blocks.d[bl->idx.d[bl->idx.n - 1]];
      const uint32_t last_clock = last->kind == BK_ITEM ? last->clock + last->len - 1 : last->clock + last->len;
      const uint32_t v = last_clock + 1;
      bool ex;
      const int32_t en = hb_entry(&b, u.clients.keys.d[ord[i]], &ex);
      if (!ex) VPUSH(clocks, 0);
      if (v > clocks.d[en]) clocks.d[en] = v;
    }
    free(ord);
    if (!err) { /* StateVector::encode over EncoderV2: everything in the rest buffer */
      wb_var(&e.rest, b.items);
      int32_t *o2 = malloc((b.items + 1) * sizeof(int32_t));
      const size_t k2 = hb_order(&b, o2);
      for (size_t i = 0; i < k2; i++) {
        wb_var(&e.rest, b.keys.d[o2[i]]);
        wb_var(&e.rest, clocks.d[o2[i]]);
      }
      free(o2);
    }
    hb_free(&b);
    VFREE(clocks);
  }
  upd_free(&u);
  if (err) {
    e2_free(&e);
    return err;
  }
  return e2_finish(&e, out, out_len);
}

/* Update::decode_v1(u).encode_v2() and Update::decode_v2(u).encode_v1() (update.rs encode_v1/
 * encode_v2 = encode_diff with an empty state vector).  Test helpers: the same document in
 * both formats.  Embed/Format values cross formats through JSON text <-> Any, which these
 * helpers do not restate (UNSUPPORTED). */
int yo_convert_update_v1_to_v2(const uint8_t *update, size_t len, uint8_t **out, size_t *out_len) {
  *out = NULL;
  *out_len = 0;
  upd_t u;
  int err = decode_update(&u, update, len);
  if (!err && u.unsupported) err = YO_ERR_UNSUPPORTED;
  enc2_t e;
  memset(&e, 0, sizeof(e));
  if (!err) {
    clist_t *cl;
    const size_t ncl = update_clients(&u, &cl);
    err = encode_blocks2(&e, cl, ncl, NULL);
    free_clients(cl, ncl);
    if (!err) ds_encode2(&e, &u.ds, u.dsv.d);
  }
  upd_free(&u);
  if (err) {
    e2_free(&e);
    return err;
  }
  return e2_finish(&e, out, out_len);
}
int yo_convert_update_v2_to_v1(const uint8_t *update, size_t len, uint8_t **out, size_t *out_len) {
  *out = NULL;
  *out_len = 0;
  upd_t u;
  int err = decode_update2(&u, update, len);
  if (!err && u.unsupported) err = YO_ERR_UNSUPPORTED;
  for (size_t i = 0; !err && i < u.blocks.n; i++)
    if (u.blocks.d[i].json_any) err = YO_ERR_UNSUPPORTED;
  wb_t w = {0};
  if (!err) {
    clist_t *cl;
    const size_t ncl = update_clients(&u, &cl);
    err = encode_blocks(&w, cl, ncl, NULL);
    free_clients(cl, ncl);
    if (!err) ds_encode(&w, &u.ds, u.dsv.d);
  }
  upd_free(&u);
  if (err) {
    free(w.d);
    return err;
  }
  return finish(&w, out, out_len);
}
