// ycompact.hip — store-based compaction on the device: a yrs Doc (GC on) applies a document's
// v1 updates in order, one transaction each, then encode_state_as_update_v1 (SURVEY §8f row 3;
// yrs/src/transaction.rs:73-85, 664-726, 828-910).  One lane per document: YATA integration is
// sequential within a document, documents are independent.
//
// Restated per transaction (update):
//   decode (walk_update: Update::decode_v1's exact errors) -> integrate the blocks in yrs'
//   order (clients descending, update.rs:169-308) with Item::repair + YATA
//   (yrs/src/block.rs:1287-1350, 482-771) -> apply_delete (transaction.rs:472-578) -> commit:
//   DeleteSet squash, GC of deleted content (gc.rs:10-66), DeleteSet::try_squash_with
//   (id_set.rs:571-598), squash of the new blocks and of split points (transaction.rs:880-910,
//   block.rs:775-799, block_store.rs:155-271).  Then blocks per client (descending) and the
//   DeleteSet built from the store in hashbrown order (id_set.rs:448-468).
//
// Device shape (documents outside it get status UNSUPPORTED; the CPU oracle covers them):
// Item contents Deleted / JSON / Binary / String / Embed / Format / Type (not WeakLink) / Any,
// GC and Skip blocks; named roots (<= 8) and nested types (ID parents) with parent_sub map
// entries; <= 8 clients; every block integrates when it arrives (no missing dependency, no
// clock gap, no partially known block) and every deleted range is known (no pending structs
// or delete sets); no String split inside a surrogate pair; per update <= 16 blocks and <= 64
// deleted ranges; the output fits the document's slot.
//
// Per-document HBM scratch (cp_words): items (I_W words), content segments (3 words: byte
// offset in the document, length / element count, next), per-client arrays of the blocks as
// they arrived (start clock, item; lookups binary-search them and walk the clock chain),
// per-update buffers, the transaction DeleteSet, branches (root and nested types) with their
// map entries (parent_sub -> current item), and a work stack for recursive deletes / GC.
#include "ycodec.h"
#include "ykernels.h"
#include "ywalk.h"

namespace ym {

constexpr uint32_t CP_MAXCL = 16, CP_MAXROOT = 8;
constexpr uint32_t CP_STAGE = 256; // per-lane LDS copy of the current update (bytes)
constexpr uint32_t CP_IS = 32, CP_IN = 28; // arrival index: one sample per 32 arrivals, 28 samples
constexpr uint32_t CP_LANES = 16;          // documents per wavefront at most (LDS sized for them)
constexpr uint32_t CNIL = 0xFFFFFFFFu;
// item words
enum : uint32_t {
  I_FWD = 0, // absorbed into (squash), else CNIL
  I_CLOCK,
  I_LEN,
  I_LEFT,
  I_RIGHT,
  I_CPREV,
  I_CNEXT,
  I_FLAGS,
  I_OC,
  I_OK,
  I_RC,
  I_RK,
  I_SEG0,
  I_SEG1,
  I_MKI,
  I_MKC,
  I_PAR, // parent branch (CNIL: TypePtr::Unknown)
  I_PSO, // parent_sub key: byte offset in the document
  I_PSL, // its length | PS_HAS (0: no parent_sub)
  I_W
};
constexpr uint32_t PS_HAS = 0x80000000u, PS_LEN = 0x7FFFFFFFu;
// Content: ItemContent ref in bits 12-15 (cp_ref); F_DELC = Deleted; F_OPQ: one clock, never
// split nor squashed (Binary / Embed / Format / Type): one segment over its content bytes,
// re-encoded by cp_opaque (a Type item keeps its own branch in I_SEG1); String / Any / JSON:
// a segment list (String: byte ranges; Any / JSON: element runs).  F_GCM: marked by the GC of
// a deleted parent type (becomes a GC struct at the end of the commit).  Bits 24-31: client.
constexpr uint32_t F_ORIGIN = 1, F_RO = 2, F_DEL = 4, F_DELC = 8, F_GC = 16, F_OPQ = 32, F_GCM = 64;
__host__ __device__ inline uint32_t cp_ref(uint32_t fl) { return (fl >> 12) & 15; }
// misc area layout (words)
enum : uint32_t {
  M_CLID = 0,                      // client ids [CP_MAXCL]
  M_HEAD = M_CLID + CP_MAXCL,      // first item in clock order 
  M_TAIL = M_HEAD + CP_MAXCL,      // last item 
  M_NBLK = M_TAIL + CP_MAXCL,      // arrived blocks 
  M_BEFORE = M_NBLK + CP_MAXCL,    // clock before the transaction 
  M_ROOTOFF = M_BEFORE + CP_MAXCL, // root name byte offset [4]
  M_ROOTLEN = M_ROOTOFF + CP_MAXROOT,
  M_ROOTBR = M_ROOTLEN + CP_MAXROOT, // its branch
  M_CBK = M_ROOTBR + CP_MAXROOT,     // client -> its arrival array (index into the count header)
  M_UE = M_CBK + CP_MAXCL,          // update DS entry clients [16] (table order)
  M_UEN = M_UE + 16,               // ranges per entry [16]
  M_HCL = M_UEN + 16,               // the count header's block clients 
  M_HCN = M_HCL + CP_MAXCL,         // their block counts (arrival capacities) 
  M_HCO = M_HCN + CP_MAXCL,         // their arrival arrays' offsets (pairs) 
  M_HNCL = M_HCO + CP_MAXCL,        // header clients
  M_CLKEND = M_HNCL + 1,            // ClientBlockList::clock of each client 
  M_IDX = M_CLKEND + CP_MAXCL,      // per client: start clock of every CP_IS-th arrival [CP_MAXCL x CP_IN]
  M_END = M_IDX + CP_MAXCL * CP_IN
};
static_assert(M_END <= 1024, "misc area");
static_assert(CP_LANES * (M_END * 4 + CP_STAGE) <= 48 * 1024, "three workgroups per CU");
// per-document counts from k_compact_count (CP_HDR words per document): blocks, deleted
// ranges, the most blocks / ranges of one update, distinct block clients (<= CP_MAXCL), and each
// client's block count (its arrival array)
enum : uint32_t { H_NB = 0, H_NR, H_MB, H_MR, H_NCL, H_OVER, H_CL = 8, H_CN = H_CL + CP_MAXCL, CP_HDR = H_CN + CP_MAXCL };
static_assert(CP_HDR == COMPACT_HDR_WORDS, "count header (ykernels.h)");
__device__ __forceinline__ uint64_t cp_words(const uint32_t *h) { // scratch words of one document
  const uint64_t items = 3ull * h[H_NB] + 2ull * h[H_NR] + 64;
  // misc, items + segments + transaction, arrivals, update buffers, branches, map entries +
  // work stack + GC marks
  return 1024 + items * (I_W + 6) + 2ull * (h[H_NB] + 8) + 9ull * h[H_MB] + 3ull * h[H_MR] + 4ull * h[H_MR] + 64 +
         4ull * (h[H_NB] + CP_MAXROOT + 8) + 6ull * items;
}
// why a document is outside the device shape (written to FastOut::path)
enum : uint32_t {
  CU_CLIENTS = 1,    // more than CP_MAXCL clients
  CU_ITEMS,          // item / segment scratch full
  CU_SURROGATE,      // String split inside a surrogate pair
  CU_TXN,            // transaction DeleteSet / merge-block list full
  CU_ARRIVALS,       // per-client arrival array full
  CU_GAP,            // clock gap: pending structs
  CU_PARTIAL,        // partially known block (integrate with an offset)
  CU_PARENT,         // (unused since round 6: nested types and parent_sub are on the device)
  CU_ROOTS,          // more than CP_MAXROOT root types
  CU_PENDING_DS,     // deleted range beyond the known state: pending delete set
  CU_PENDING,        // missing dependency: pending structs
  CU_UPDATE_SHAPE,   // update over DS_SMALL delete-set entries, or Doc / Move / WeakLink content
  CU_OUTPUT          // output over the document's slot
};

struct CDoc {
  const uint8_t *p;  // the document's bytes
  const uint8_t *up; // the current update's bytes (an LDS copy when it fits the lane's stage)
  uint32_t uoff;     // its offset in the document
  uint32_t *it, *sg, *cb, *m;
  uint32_t *ubr, *ub, *stk, *ur, *mb; // update blocks (stream order, integration order), stack,
                                      // DS ranges, merge blocks
  uint32_t *tx;                       // transaction DeleteSet (client index, start, end), cap_i
  uint32_t *bt, *me, *wk, *gm;        // branches (BR_W), map entries (ME_W), work stack, GC marks
  const uint32_t *h;                  // the document's count header
  uint32_t ni, cap_i, ns, cap_s, mB, mR;
  uint32_t nbr, cap_b, nme, ngm;
  uint32_t ncl, nroot, nub, nur, nue, nt, nm;
  uint32_t gen_i, gen_c;
  int st;      // status (first error / unsupported)
  uint32_t why; // CU_* reason of an E_UNSUPPORTED status (FastOut::path, diagnostics)
  __device__ uint32_t &I(uint32_t x, uint32_t f) { return it[(size_t)x * I_W + f]; }
  __device__ uint32_t cl_of(uint32_t x) { return I(x, I_FLAGS) >> 24; }
};

__device__ void cp_unsup(CDoc &D, uint32_t why) {
  D.st = E_UNSUPPORTED;
  D.why = why;
}

// ------------------------------------------------------------------ clients, lookups
__device__ int cp_cl_find(CDoc &D, uint32_t client) {
  for (uint32_t i = 0; i < D.ncl; i++)
    if (D.m[M_CLID + i] == client) return (int)i;
  return -1;
}
__device__ int cp_cl_add(CDoc &D, uint32_t client) { // BlockStore::get_client_blocks_mut (first push)
  int c = cp_cl_find(D, client);
  if (c >= 0) return c;
  if (D.ncl == CP_MAXCL) {
    cp_unsup(D, CU_CLIENTS);
    return -1;
  }
  uint32_t k = 0;
  while (k < D.m[M_HNCL] && D.m[M_HCL + k] != client) k++;
  if (k == D.m[M_HNCL]) {
    cp_unsup(D, CU_ARRIVALS);
    return -1;
  }
  c = (int)D.ncl++;
  D.m[M_CLID + c] = client;
  D.m[M_CBK + c] = k;
  D.m[M_HEAD + c] = D.m[M_TAIL + c] = CNIL;
  D.m[M_NBLK + c] = 0;
  D.m[M_BEFORE + c] = 0;
  D.m[M_CLKEND + c] = 0;
  return c;
}
__device__ uint32_t cp_fwd(CDoc &D, uint32_t x) {
  for (uint32_t g = D.ni; D.I(x, I_FWD) != CNIL && g; g--) x = D.I(x, I_FWD);
  return x;
}
__device__ uint32_t cp_clock(CDoc &D, int c) { // ClientBlockList::clock (kept by cp_push)
  return c < 0 ? 0 : D.m[M_CLKEND + c];
}
// find_pivot: the cell (item or GC) containing clock, or CNIL
__device__ uint32_t cp_cell(CDoc &D, int c, uint32_t clock) {
  if (c < 0) return CNIL;
  const uint32_t n = D.m[M_NBLK + c];
  const uint32_t *a = D.cb + 2ull * D.m[M_HCO + D.m[M_CBK + c]];
  if (!n || D.m[M_IDX + c * CP_IN] > clock) return CNIL;
  // the client's last item first (two loads): an insert's origin is most often its client's
  // latest text, and a clock at or past that item's start is in it or in no cell
  const uint32_t t = D.m[M_TAIL + c];
  if (t != CNIL) {
    const uint32_t t0 = D.I(t, I_CLOCK), tl = D.I(t, I_LEN);
    if (clock >= t0) return clock - t0 < tl ? t : CNIL;
  }
  // last arrived block starting <= clock: the sampled starts in LDS narrow the search of the
  // arrival array in HBM to one run of CP_IS arrivals (or to the arrivals past the samples)
  const uint32_t *ix = D.m + M_IDX + c * CP_IN;
  const uint32_t ns = (n + CP_IS - 1) / CP_IS < CP_IN ? (n + CP_IS - 1) / CP_IS : CP_IN;
  uint32_t s0 = 0, s1 = ns - 1;
  while (s0 < s1) {
    const uint32_t mid = (s0 + s1 + 1) / 2;
    if (ix[mid] <= clock) s0 = mid;
    else s1 = mid - 1;
  }
  uint32_t lo = s0 * CP_IS, hi = s0 + 1 < ns ? (s0 + 1) * CP_IS - 1 : n - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) / 2;
    if (a[2 * mid] <= clock) lo = mid;
    else hi = mid - 1;
  }
  uint32_t x = cp_fwd(D, a[2 * lo + 1]);
  for (uint32_t g = D.ni; x != CNIL && clock >= D.I(x, I_CLOCK) + D.I(x, I_LEN); x = D.I(x, I_CNEXT))
    if (g-- == 0) return CNIL;
  if (x == CNIL || clock < D.I(x, I_CLOCK)) return CNIL;
  return x;
}
__device__ uint32_t cp_get_item(CDoc &D, uint32_t client, uint32_t clock) { // BlockStore::get_item
  const uint32_t x = cp_cell(D, cp_cl_find(D, client), clock);
  return (x == CNIL || (D.I(x, I_FLAGS) & F_GC)) ? CNIL : x;
}

// ------------------------------------------------------------------ content
__device__ uint32_t cp_new_item(CDoc &D) {
  if (D.ni == D.cap_i) {
    cp_unsup(D, CU_ITEMS);
    return CNIL;
  }
  const uint32_t x = D.ni++;
  for (uint32_t f = 0; f < I_W; f++) D.I(x, f) = 0;
  D.I(x, I_FWD) = D.I(x, I_LEFT) = D.I(x, I_RIGHT) = D.I(x, I_CPREV) = D.I(x, I_CNEXT) = CNIL;
  D.I(x, I_SEG0) = D.I(x, I_SEG1) = D.I(x, I_PAR) = CNIL;
  return x;
}
// segment words: byte offset in the document, length | SEG_ASCII (every char one byte: UTF-16
// offsets are byte offsets), next
constexpr uint32_t SEG_ASCII = 0x80000000u, SEG_LEN = 0x7FFFFFFFu;
__device__ uint32_t cp_new_seg(CDoc &D, uint32_t off, uint32_t n) {
  if (D.ns == D.cap_s) {
    cp_unsup(D, CU_ITEMS);
    return CNIL;
  }
  const uint32_t s = D.ns++;
  D.sg[3 * s] = off;
  D.sg[3 * s + 1] = n;
  D.sg[3 * s + 2] = CNIL;
  return s;
}
// ItemContent::splice(off, Utf16) of a String (block.rs:1837-1879, split_str :1483-1502): the
// item keeps [0, off) (a char is never cut: the UTF-16 offset maps to the next char boundary;
// landing inside a surrogate pair is outside the device shape); returns the right part's
// first segment.  Its UTF-16 length is the item's minus off: an item's length equals its
// content's UTF-16 length on the device (the surrogate case above is the only exception).
__device__ uint32_t cp_str_split(CDoc &D, uint32_t x, uint32_t off) {
  uint32_t u = 0, s = D.I(x, I_SEG0);
  while (s != CNIL) {
    const uint32_t lw = D.sg[3 * s + 1], n = lw & SEG_LEN;
    uint32_t i = 0;
    if (lw & SEG_ASCII) {
      i = off - u < n ? off - u : n;
      u += i;
    } else {
      const uint8_t *b = D.p + D.sg[3 * s];
      while (i < n && u < off) {
        const uint32_t ch = utf8_next(b, n, i);
        u += ch_len16(ch);
      }
    }
    if (u >= off) {
      if (u != off) {
        cp_unsup(D, CU_SURROGATE); // split inside a surrogate pair
        return CNIL;
      }
      uint32_t r;
      if (i == n) { // boundary at the end of segment s
        r = D.sg[3 * s + 2];
        D.sg[3 * s + 2] = CNIL;
        D.I(x, I_SEG1) = s;
      } else {
        r = cp_new_seg(D, D.sg[3 * s] + i, (n - i) | (lw & SEG_ASCII));
        if (r == CNIL) return CNIL;
        D.sg[3 * r + 2] = D.sg[3 * s + 2];
        D.sg[3 * s + 1] = i | (lw & SEG_ASCII);
        D.sg[3 * s + 2] = CNIL;
        D.I(x, I_SEG1) = s;
      }
      return r;
    }
    s = D.sg[3 * s + 2];
  }
  D.st = E_PANIC; // offset past the content: yrs' splice unwraps None
  return CNIL;
}
// ItemContent::splice(off) of an Any / JSON list (block.rs:1837-1879): element runs, split
// inside a run at the byte offset of its (off - u)-th element (Any values: any_skip; JSON:
// strings); returns the right part's first segment
__device__ uint32_t cp_el_split(CDoc &D, uint32_t x, uint32_t off, bool any) {
  uint32_t u = 0, s = D.I(x, I_SEG0);
  while (s != CNIL) {
    const uint32_t n = D.sg[3 * s + 1];
    if (off - u <= n) {
      const uint32_t k = off - u;
      uint32_t r;
      if (k == n) { // boundary at the end of run s
        r = D.sg[3 * s + 2];
        D.sg[3 * s + 2] = CNIL;
      } else {
        Cur c{D.p, 0xFFFFFFFFu, D.sg[3 * s]};
        for (uint32_t q = 0; q < k; q++) {
          if (any) {
            any_skip(c);
          } else {
            uint32_t v;
            bool cn;
            rd_var_u32(c, v, cn);
            c.i += v;
          }
        }
        r = cp_new_seg(D, c.i, n - k);
        if (r == CNIL) return CNIL;
        D.sg[3 * r + 2] = D.sg[3 * s + 2];
        D.sg[3 * s + 1] = k;
        D.sg[3 * s + 2] = CNIL;
      }
      D.I(x, I_SEG1) = s;
      return r;
    }
    u += n;
    s = D.sg[3 * s + 2];
  }
  D.st = E_PANIC;
  return CNIL;
}

// ------------------------------------------------------------------ branches (types) and maps
// A branch: root type (name in the misc root table) or the nested type of a Type item; its
// sequence start and its map (parent_sub -> current item: entries in insertion order).
enum : uint32_t { B_START = 0, B_ITEM, B_MAP, B_ROOT, BR_W };
enum : uint32_t { E_KOFF = 0, E_KLEN, E_VAL, E_NEXT, ME_W };
__device__ uint32_t cp_new_branch(CDoc &D, uint32_t item, uint32_t root) {
  if (D.nbr == D.cap_b) {
    cp_unsup(D, CU_ITEMS);
    return CNIL;
  }
  uint32_t *b = D.bt + (size_t)BR_W * D.nbr;
  b[B_START] = CNIL;
  b[B_ITEM] = item;
  b[B_MAP] = CNIL;
  b[B_ROOT] = root;
  return D.nbr++;
}
__device__ uint32_t &cp_bw(CDoc &D, uint32_t b, uint32_t f) { return D.bt[(size_t)BR_W * b + f]; }
// the map entry of x's parent_sub key in branch b (CNIL: none)
__device__ uint32_t cp_map_entry(CDoc &D, uint32_t b, uint32_t x) {
  const uint32_t ko = D.I(x, I_PSO), kn = D.I(x, I_PSL) & PS_LEN;
  for (uint32_t e = cp_bw(D, b, B_MAP); e != CNIL; e = D.me[ME_W * e + E_NEXT])
    if (D.me[ME_W * e + E_KLEN] == kn && bytes_eq(D.p + D.me[ME_W * e + E_KOFF], D.p + ko, kn)) return e;
  return CNIL;
}
__device__ uint32_t cp_map_get(CDoc &D, uint32_t b, uint32_t x) {
  const uint32_t e = cp_map_entry(D, b, x);
  return e == CNIL ? CNIL : D.me[ME_W * e + E_VAL];
}
__device__ void cp_map_set(CDoc &D, uint32_t b, uint32_t x, uint32_t v) { // key of x -> v
  uint32_t e = cp_map_entry(D, b, x);
  if (e == CNIL) {
    if (D.nme == D.cap_i) {
      cp_unsup(D, CU_ITEMS);
      return;
    }
    e = D.nme++;
    D.me[ME_W * e + E_KOFF] = D.I(x, I_PSO);
    D.me[ME_W * e + E_KLEN] = D.I(x, I_PSL) & PS_LEN;
    D.me[ME_W * e + E_NEXT] = CNIL;
    uint32_t *link = &cp_bw(D, b, B_MAP);
    while (*link != CNIL) link = &D.me[ME_W * *link + E_NEXT];
    *link = e;
  }
  D.me[ME_W * e + E_VAL] = v;
}
// the leftmost item of x's key in branch b (the YATA scan start / relink point of a map entry)
__device__ uint32_t cp_map_first(CDoc &D, uint32_t b, uint32_t x) {
  uint32_t o = cp_map_get(D, b, x);
  for (uint32_t g = D.ni; o != CNIL && D.I(o, I_LEFT) != CNIL && g; g--) o = D.I(o, I_LEFT);
  return o;
}

// ItemPtr::splice + BlockStore::split_block (block.rs:435-478, block_store.rs:456-475)
__device__ uint32_t cp_split(CDoc &D, uint32_t x, uint32_t off) {
  if (off == 0) return CNIL;
  const uint32_t r = cp_new_item(D);
  if (r == CNIL) return CNIL;
  const uint32_t fl = D.I(x, I_FLAGS);
  if (fl & F_DELC) {
    D.I(r, I_LEN) = D.I(x, I_LEN) - off;
  } else if (fl & F_OPQ) { // one-clock content: splice returns None, yrs unwraps
    D.st = E_PANIC;
    return CNIL;
  } else {
    const uint32_t seg1 = D.I(x, I_SEG1); // the right part ends where the item did
    const uint32_t ref = cp_ref(fl);
    const uint32_t rs = ref == 4 ? cp_str_split(D, x, off) : cp_el_split(D, x, off, ref == 8);
    if (D.st) return CNIL;
    D.I(r, I_SEG0) = rs;
    // the split segment was the last one: the new right segment is the last; else the old last
    D.I(r, I_SEG1) = rs == CNIL ? CNIL : D.I(x, I_SEG1) == seg1 ? rs : seg1;
    D.I(r, I_LEN) = D.I(x, I_LEN) - off;
  }
  const uint32_t c = fl >> 24;
  D.I(r, I_CLOCK) = D.I(x, I_CLOCK) + off;
  D.I(r, I_FLAGS) = (fl & ~(uint32_t)F_ORIGIN) | F_ORIGIN;
  D.I(r, I_OC) = D.m[M_CLID + c];
  D.I(r, I_OK) = D.I(x, I_CLOCK) + off - 1;
  D.I(r, I_RC) = D.I(x, I_RC);
  D.I(r, I_RK) = D.I(x, I_RK);
  D.I(r, I_PAR) = D.I(x, I_PAR);
  D.I(r, I_PSO) = D.I(x, I_PSO);
  D.I(r, I_PSL) = D.I(x, I_PSL);
  D.I(x, I_LEN) = off;
  // list links (the right part of a parent's current map value becomes the value)
  const uint32_t xr = D.I(x, I_RIGHT);
  if ((D.I(x, I_PSL) & PS_HAS) && xr == CNIL && D.I(x, I_PAR) != CNIL) cp_map_set(D, D.I(x, I_PAR), x, r);
  D.I(r, I_LEFT) = x;
  D.I(r, I_RIGHT) = xr;
  if (xr != CNIL) D.I(xr, I_LEFT) = r;
  D.I(x, I_RIGHT) = r;
  // clock chain
  const uint32_t xn = D.I(x, I_CNEXT);
  D.I(r, I_CPREV) = x;
  D.I(r, I_CNEXT) = xn;
  if (xn != CNIL) D.I(xn, I_CPREV) = r;
  else D.m[M_TAIL + c] = r;
  D.I(x, I_CNEXT) = r;
  return r;
}
__device__ uint32_t cp_clean_start(CDoc &D, uint32_t client, uint32_t clock) {
  const uint32_t x = cp_get_item(D, client, clock);
  if (x == CNIL) return CNIL;
  const uint32_t off = clock - D.I(x, I_CLOCK);
  return off == 0 ? x : cp_split(D, x, off);
}
__device__ uint32_t cp_clean_end(CDoc &D, uint32_t client, uint32_t clock) {
  const uint32_t x = cp_get_item(D, client, clock);
  if (x == CNIL) return CNIL;
  const uint32_t off = clock - D.I(x, I_CLOCK);
  if (off + 1 < D.I(x, I_LEN)) cp_split(D, x, off + 1);
  return x;
}

// ------------------------------------------------------------------ transaction
__device__ void cp_txn_insert(CDoc &D, uint32_t c, uint32_t s, uint32_t e) {
  if (D.nt && D.tx[3 * (D.nt - 1)] == c && D.tx[3 * (D.nt - 1) + 2] == s) { // IdRange::push joins
    D.tx[3 * (D.nt - 1) + 2] = e;
    return;
  }
  if (D.nt == D.cap_i) {
    cp_unsup(D, CU_TXN);
    return;
  }
  D.tx[3 * D.nt] = c;
  D.tx[3 * D.nt + 1] = s;
  D.tx[3 * D.nt + 2] = e;
  D.nt++;
}
__device__ void cp_merge_block(CDoc &D, uint32_t c, uint32_t clock);
// TransactionMut::delete (transaction.rs:579-662): the item; a Type's children (its sequence's
// live items, then every current map value) depth first, in that order (an explicit stack);
// a child already deleted goes to merge_blocks
__device__ bool cp_delete(CDoc &D, uint32_t x0) {
  uint32_t sp = 0;
  bool result = false, top = true;
  D.wk[sp++] = x0;
  while (sp && !D.st) {
    const uint32_t x = D.wk[--sp];
    uint32_t &fl = D.I(x, I_FLAGS);
    if (fl & F_DEL) {
      if (!top) cp_merge_block(D, fl >> 24, D.I(x, I_CLOCK));
      top = false;
      continue;
    }
    if (top) result = true;
    top = false;
    fl |= F_DEL;
    cp_txn_insert(D, fl >> 24, D.I(x, I_CLOCK), D.I(x, I_CLOCK) + D.I(x, I_LEN));
    if (cp_ref(fl) != 7 || (fl & F_DELC)) continue;
    const uint32_t b = D.I(x, I_SEG1);
    uint32_t n = 0;
    for (uint32_t p = cp_bw(D, b, B_START), g = D.ni; p != CNIL && g; p = D.I(p, I_RIGHT), g--)
      n += !(D.I(p, I_FLAGS) & F_DEL);
    for (uint32_t e = cp_bw(D, b, B_MAP); e != CNIL; e = D.me[ME_W * e + E_NEXT]) n++;
    if (sp + n > D.cap_i) {
      cp_unsup(D, CU_ITEMS);
      return result;
    }
    uint32_t k = sp + n; // children popped in order: the first on top
    for (uint32_t p = cp_bw(D, b, B_START), g = D.ni; p != CNIL && g; p = D.I(p, I_RIGHT), g--)
      if (!(D.I(p, I_FLAGS) & F_DEL)) D.wk[--k] = p;
    for (uint32_t e = cp_bw(D, b, B_MAP); e != CNIL; e = D.me[ME_W * e + E_NEXT]) D.wk[--k] = D.me[ME_W * e + E_VAL];
    sp += n;
  }
  return result;
}
__device__ void cp_merge_block(CDoc &D, uint32_t c, uint32_t clock) {
  if (D.nm == 2 * D.mR + 2) {
    cp_unsup(D, CU_TXN);
    return;
  }
  D.mb[2 * D.nm] = c;
  D.mb[2 * D.nm + 1] = clock;
  D.nm++;
}

// ------------------------------------------------------------------ integrate (block.rs:482-771)
__device__ bool cp_same_origin(CDoc &D, uint32_t a, uint32_t b) {
  const uint32_t fa = D.I(a, I_FLAGS) & F_ORIGIN, fb = D.I(b, I_FLAGS) & F_ORIGIN;
  return fa == fb && (!fa || (D.I(a, I_OC) == D.I(b, I_OC) && D.I(a, I_OK) == D.I(b, I_OK)));
}
__device__ bool cp_same_ro(CDoc &D, uint32_t a, uint32_t b) {
  const uint32_t fa = D.I(a, I_FLAGS) & F_RO, fb = D.I(b, I_FLAGS) & F_RO;
  return fa == fb && (!fa || (D.I(a, I_RC) == D.I(b, I_RC) && D.I(a, I_RK) == D.I(b, I_RK)));
}
// the new item x is repaired (left / right / parent branch set); links it into its parent's
// sequence or map entry (block.rs:482-771).  Returns true when x must be deleted right after
// (its parent type is deleted, or it is not the current value of its map key).
__device__ bool cp_integrate(CDoc &D, uint32_t x) {
  const uint32_t par = D.I(x, I_PAR);
  uint32_t left = D.I(x, I_LEFT), right = D.I(x, I_RIGHT);
  const bool rnull_or_left = right == CNIL || D.I(right, I_LEFT) != CNIL;
  const bool left_other = left != CNIL && D.I(left, I_RIGHT) != right;
  if ((left == CNIL && rnull_or_left) || left_other) {
    uint32_t o = left != CNIL                  ? D.I(left, I_RIGHT)
                 : (D.I(x, I_PSL) & PS_HAS) ? cp_map_first(D, par, x)
                                            : cp_bw(D, par, B_START);
    uint32_t nl = left;
    const uint32_t gi = ++D.gen_i;
    uint32_t gc = ++D.gen_c;
    const uint32_t xcl = D.m[M_CLID + D.cl_of(x)];
    uint32_t guard = D.ni; // every item at most once: a broken list ends here, not in a hang
    while (o != CNIL && o != D.I(x, I_RIGHT)) {
      if (guard-- == 0) {
        cp_unsup(D, CU_ITEMS);
        return false;
      }
      D.I(o, I_MKI) = gi;
      D.I(o, I_MKC) = gc;
      if (cp_same_origin(D, x, o)) {
        if (D.m[M_CLID + D.cl_of(o)] < xcl) {
          nl = o;
          gc = ++D.gen_c;
        } else if (cp_same_ro(D, x, o)) {
          break;
        }
      } else {
        const uint32_t op = (D.I(o, I_FLAGS) & F_ORIGIN) ? cp_get_item(D, D.I(o, I_OC), D.I(o, I_OK)) : CNIL;
        if (op == CNIL || D.I(op, I_MKI) != gi) break;
        if (D.I(op, I_MKC) != gc) {
          nl = o;
          gc = ++D.gen_c;
        }
      }
      o = D.I(o, I_RIGHT);
    }
    D.I(x, I_LEFT) = nl;
  }
  left = D.I(x, I_LEFT);
  if (!(D.I(x, I_PSL) & PS_HAS) && left != CNIL) { // parent_sub from the neighbours
    const uint32_t src = (D.I(left, I_PSL) & PS_HAS) ? left : D.I(x, I_RIGHT);
    if (src != CNIL) {
      D.I(x, I_PSO) = D.I(src, I_PSO);
      D.I(x, I_PSL) = D.I(src, I_PSL);
    }
  }
  const bool psub = D.I(x, I_PSL) & PS_HAS;
  if (left != CNIL) {
    D.I(x, I_RIGHT) = D.I(left, I_RIGHT);
    D.I(left, I_RIGHT) = x;
  } else if (psub) {
    D.I(x, I_RIGHT) = cp_map_first(D, par, x);
  } else {
    D.I(x, I_RIGHT) = cp_bw(D, par, B_START);
    cp_bw(D, par, B_START) = x;
  }
  right = D.I(x, I_RIGHT);
  if (right != CNIL) {
    D.I(right, I_LEFT) = x;
  } else if (psub) { // the key's current value; the previous one is deleted
    cp_map_set(D, par, x, x);
    if (left != CNIL) cp_delete(D, left);
  }
  if (D.I(x, I_FLAGS) & F_DELC) { // ItemContent::Deleted
    D.I(x, I_FLAGS) |= F_DEL;
    cp_txn_insert(D, D.cl_of(x), D.I(x, I_CLOCK), D.I(x, I_CLOCK) + D.I(x, I_LEN));
  }
  if (cp_ref(D.I(x, I_FLAGS)) == 7) { // ItemContent::Type: its branch
    const uint32_t b = cp_new_branch(D, x, CNIL);
    if (b == CNIL) return false;
    D.I(x, I_SEG1) = b;
  }
  const uint32_t pit = cp_bw(D, par, B_ITEM);
  return (pit != CNIL && (D.I(pit, I_FLAGS) & F_DEL)) || (psub && D.I(x, I_RIGHT) != CNIL);
}
// appends a cell to its client's clock chain and arrival array
__device__ void cp_push(CDoc &D, int c, uint32_t x) {
  const uint32_t t = D.m[M_TAIL + c];
  D.I(x, I_CPREV) = t;
  D.I(x, I_CNEXT) = CNIL;
  if (t != CNIL) D.I(t, I_CNEXT) = x;
  else D.m[M_HEAD + c] = x;
  D.m[M_TAIL + c] = x;
  const uint32_t n = D.m[M_NBLK + c];
  const uint32_t k = D.m[M_CBK + c];
  if (n == D.m[M_HCN + k]) {
    cp_unsup(D, CU_ARRIVALS);
    return;
  }
  uint32_t *a = D.cb + 2ull * D.m[M_HCO + k];
  const uint32_t clock = D.I(x, I_CLOCK);
  a[2 * n] = clock;
  a[2 * n + 1] = x;
  if (n % CP_IS == 0 && n / CP_IS < CP_IN) D.m[M_IDX + c * CP_IN + n / CP_IS] = clock;
  D.m[M_CLKEND + c] = clock + D.I(x, I_LEN);
  D.m[M_NBLK + c] = n + 1;
}

// ------------------------------------------------------------------ squash (block.rs:775-799)
__device__ bool cp_try_squash(CDoc &D, uint32_t l, uint32_t r) { // squash r into l
  const uint32_t fl = D.I(l, I_FLAGS), fr = D.I(r, I_FLAGS);
  if ((fl & F_GC) || (fr & F_GC)) return false;
  const uint32_t c = fl >> 24;
  if (!(D.I(l, I_CLOCK) + D.I(l, I_LEN) == D.I(r, I_CLOCK) && (fr & F_ORIGIN) && D.I(r, I_OC) == D.m[M_CLID + c] &&
        D.I(r, I_OK) == D.I(l, I_CLOCK) + D.I(l, I_LEN) - 1 && cp_same_ro(D, l, r) && D.I(l, I_RIGHT) == r &&
        (fl & F_DEL) == (fr & F_DEL) && cp_ref(fl) == cp_ref(fr) && !((fl | fr) & F_OPQ)))
    return false; // (ItemContent::try_squash, block.rs:1884-1906: String, Any, JSON, Deleted)
  if (!(fl & F_DELC)) { // segment lists concatenated
    D.sg[3 * D.I(l, I_SEG1) + 2] = D.I(r, I_SEG0);
    D.I(l, I_SEG1) = D.I(r, I_SEG1);
  }
  D.I(l, I_LEN) += D.I(r, I_LEN);
  const uint32_t rr = D.I(r, I_RIGHT);
  if (rr != CNIL) D.I(rr, I_LEFT) = l;
  D.I(l, I_RIGHT) = rr;
  // the map's current value was r: now l (s_fix_map)
  if ((D.I(r, I_PSL) & PS_HAS) && D.I(r, I_PAR) != CNIL && cp_map_get(D, D.I(r, I_PAR), r) == r)
    cp_map_set(D, D.I(r, I_PAR), r, l);
  return true;
}
// unlinks r (squashed into its clock predecessor l) from the clock chain
__device__ void cp_unchain(CDoc &D, uint32_t l, uint32_t r) {
  const uint32_t rn = D.I(r, I_CNEXT);
  D.I(l, I_CNEXT) = rn;
  if (rn != CNIL) D.I(rn, I_CPREV) = l;
  else D.m[M_TAIL + D.cl_of(l)] = l;
  D.I(r, I_FWD) = l;
}
// ClientBlockList::squash_left (block_store.rs:243-271): r into its clock predecessor
__device__ void cp_squash_left(CDoc &D, uint32_t r) {
  const uint32_t l = D.I(r, I_CPREV);
  if (l == CNIL) return;
  const bool gl = D.I(l, I_FLAGS) & F_GC, gr = D.I(r, I_FLAGS) & F_GC;
  if (gl && gr) {
    D.I(l, I_LEN) += D.I(r, I_LEN);
  } else if (gl || gr || !cp_try_squash(D, l, r)) {
    return;
  }
  cp_unchain(D, l, r);
}

// ------------------------------------------------------------------ commit (transaction.rs:828-910)
// ItemContent::gc of a Type (block.rs:1907-1926): every item of its sequence and of its map
// entries' chains (current value leftwards) gets Item::gc(parent_gc = true): a deleted one is
// marked (and its own type's children visited); the branch is emptied.  Work stack of branches.
__device__ void cp_gc_content(CDoc &D, uint32_t x0) {
  const uint32_t f0 = D.I(x0, I_FLAGS);
  if (cp_ref(f0) != 7 || (f0 & (F_DELC | F_GC)) || D.I(x0, I_SEG1) == CNIL) return;
  uint32_t sp = 0;
  D.wk[sp++] = D.I(x0, I_SEG1);
  auto visit = [&](uint32_t p) {
    uint32_t &fl = D.I(p, I_FLAGS);
    if ((fl & F_GC) || !(fl & F_DEL)) return;
    if (cp_ref(fl) == 7 && !(fl & F_DELC) && D.I(p, I_SEG1) != CNIL) {
      if (sp == D.cap_i) {
        cp_unsup(D, CU_ITEMS);
        return;
      }
      D.wk[sp++] = D.I(p, I_SEG1);
      D.I(p, I_SEG1) = CNIL; // (visited once)
    }
    if (!(fl & F_GCM)) {
      fl |= F_GCM;
      if (D.ngm < D.cap_i) D.gm[D.ngm++] = p;
      else cp_unsup(D, CU_ITEMS);
    }
  };
  while (sp && !D.st) {
    const uint32_t b = D.wk[--sp];
    for (uint32_t p = cp_bw(D, b, B_START), g = D.ni; p != CNIL && g; g--) {
      const uint32_t nx = D.I(p, I_RIGHT);
      visit(p);
      p = nx;
    }
    for (uint32_t e = cp_bw(D, b, B_MAP); e != CNIL; e = D.me[ME_W * e + E_NEXT])
      for (uint32_t p = D.me[ME_W * e + E_VAL], g = D.ni; p != CNIL && g; g--) {
        const uint32_t nx = D.I(p, I_LEFT);
        visit(p);
        p = nx;
      }
    cp_bw(D, b, B_START) = CNIL;
    cp_bw(D, b, B_MAP) = CNIL;
  }
}
__device__ void cp_commit(CDoc &D) {
  // 1. DeleteSet squash per client: sort by (client, start), join overlapping / adjacent
  for (uint32_t i = 1; i < D.nt; i++) {
    const uint32_t c = D.tx[3 * i], s = D.tx[3 * i + 1], e = D.tx[3 * i + 2];
    uint32_t j = i;
    while (j > 0 && (D.tx[3 * (j - 1)] > c || (D.tx[3 * (j - 1)] == c && D.tx[3 * (j - 1) + 1] > s))) {
      for (uint32_t f = 0; f < 3; f++) D.tx[3 * j + f] = D.tx[3 * (j - 1) + f];
      j--;
    }
    D.tx[3 * j] = c;
    D.tx[3 * j + 1] = s;
    D.tx[3 * j + 2] = e;
  }
  uint32_t k = 0;
  for (uint32_t i = 0; i < D.nt; i++) {
    const uint32_t c = D.tx[3 * i], s = D.tx[3 * i + 1], e = D.tx[3 * i + 2];
    if (k && D.tx[3 * (k - 1)] == c && s <= D.tx[3 * (k - 1) + 2]) {
      if (e > D.tx[3 * (k - 1) + 2]) D.tx[3 * (k - 1) + 2] = e;
      continue;
    }
    D.tx[3 * k] = c;
    D.tx[3 * k + 1] = s;
    D.tx[3 * k + 2] = e;
    k++;
  }
  D.nt = k;
  // 4. GC (gc.rs:10-66): deleted content in the ranges -> Deleted(len); a deleted type's
  //    descendants that are deleted are marked and become GC structs after the loop
  D.ngm = 0;
  for (uint32_t i = D.nt; i-- > 0 && !D.st;) {
    const int c = (int)D.tx[3 * i];
    const uint32_t rs = D.tx[3 * i + 1], re = D.tx[3 * i + 2];
    uint32_t start = rs;
    for (uint32_t x = cp_cell(D, c, rs); x != CNIL; x = D.I(x, I_CNEXT)) {
      start += D.I(x, I_LEN);
      if (start > re) break;
      uint32_t &fl = D.I(x, I_FLAGS);
      if (!(fl & F_GC) && (fl & F_DEL)) { // Item::gc(collector, false)
        cp_gc_content(D, x);
        fl = (fl & ~(F_OPQ | 0xF000u)) | F_DELC | (1u << 12);
        D.I(x, I_SEG0) = D.I(x, I_SEG1) = CNIL;
      }
    }
  }
  for (uint32_t k = 0; k < D.ngm; k++) { // collect_all_marked: GC structs
    const uint32_t x = D.gm[k];
    uint32_t &fl = D.I(x, I_FLAGS);
    fl &= ~F_GCM;
    if (!(fl & F_GC) && (fl & F_DEL)) {
      fl = F_GC | (fl & 0xFF000000u);
      D.I(x, I_SEG0) = D.I(x, I_SEG1) = CNIL;
    }
  }
  // 5. DeleteSet::try_squash_with (id_set.rs:571-598)
  for (uint32_t i = D.nt; i-- > 0;) {
    const int c = (int)D.tx[3 * i];
    const uint32_t rs = D.tx[3 * i + 1], re = D.tx[3 * i + 2];
    const uint32_t head = D.m[M_HEAD + c];
    uint32_t p = cp_cell(D, c, re - 1);
    if (p == CNIL) p = head; // find_pivot(..).unwrap_or_default() = index 0
    uint32_t si = D.I(p, I_CNEXT) != CNIL ? D.I(p, I_CNEXT) : p; // min(len - 1, pivot + 1)
    // collect [lo..hi] walking left while the block starts at or after the range
    uint32_t hi = CNIL, lo = CNIL;
    while (D.I(si, I_CPREV) != CNIL && D.I(si, I_CLOCK) >= rs) {
      if (hi == CNIL) hi = si;
      lo = si;
      si = D.I(si, I_CPREV);
    }
    if (hi == CNIL) continue;
    // squash_left_range_compaction: pairs (prev, x) from hi down to lo
    uint32_t x = hi;
    for (;;) {
      const uint32_t prev = D.I(x, I_CPREV);
      const bool last = x == lo;
      cp_squash_left(D, x);
      if (last) break;
      x = prev;
    }
  }
  // 6. squash the blocks added by the transaction with their left neighbours
  for (uint32_t c = 0; c < D.ncl; c++) {
    const uint32_t before = D.m[M_BEFORE + c];
    if (before == cp_clock(D, (int)c)) continue;
    // from the last block down to the one holding `before` (find_pivot), index >= 1
    const uint32_t stop = cp_cell(D, (int)c, before);
    uint32_t x = D.m[M_TAIL + c];
    while (x != CNIL && D.I(x, I_CPREV) != CNIL) {
      const uint32_t prev = D.I(x, I_CPREV);
      cp_squash_left(D, x);
      if (x == stop) break;
      x = prev;
    }
  }
  // 7. merge_blocks
  for (uint32_t i = 0; i < D.nm; i++) {
    const uint32_t x = cp_cell(D, (int)D.mb[2 * i], D.mb[2 * i + 1]);
    if (x == CNIL) continue;
    if (D.I(x, I_CNEXT) != CNIL) cp_squash_left(D, D.I(x, I_CNEXT));
    else if (D.I(x, I_CPREV) != CNIL) cp_squash_left(D, x);
  }
}

// ------------------------------------------------------------------ decode sink
struct CpSink {
  CDoc *D;
  const uint8_t *p;
  uint32_t ds_client, ds_left, nent;
  bool over; // beyond the per-update buffers: outside the device shape
  __device__ void on_section(uint32_t) {}
  __device__ int on_block(uint32_t client, uint32_t clock, const BlockInfo &bi, uint32_t bpos, uint32_t) {
    // (Doc / Move contents are outside the device shape; WeakLink types: cp_block)
    if (bi.kind == BK_ITEM && (bi.ref == 9 || bi.ref >= 10)) over = true;
    if (D->nub == D->mB) {
      over = true;
      return 0;
    }
    uint32_t *b = D->ubr + 4 * D->nub++;
    b[0] = client;
    b[1] = clock;
    b[2] = bpos;
    b[3] = bi.len;
    return 0;
  }
  __device__ int on_ds_begin(uint32_t) { return 0; }
  __device__ int on_ds_entry(uint32_t client, uint32_t nr) {
    ds_client = client;
    if (nent == DS_SMALL) over = true;
    else {
      D->m[M_UE + nent] = client;
      D->m[M_UEN + nent] = nr;
      nent++;
    }
    return 0;
  }
  __device__ void on_ds_range(uint32_t s, uint32_t e) {
    if (D->nur == D->mR) {
      over = true;
      return;
    }
    uint32_t *r = D->ur + 3 * D->nur++;
    r[0] = ds_client;
    r[1] = s;
    r[2] = e;
  }
  __device__ int on_ds_done() { return 0; }
};

// one block of the update (Update::integrate's loop body, update.rs:205-262): 0 = done
// (integrated or skipped), 1 = a dependency on client `dep` is missing, -1 = stop (D.st)
__device__ int cp_block(CDoc &D, const uint32_t *ub, uint32_t &dep) {
  const uint32_t client = ub[0], clock = ub[1], bpos = ub[2], len = ub[3];
  const uint8_t info = D.up[bpos]; // bpos: within the current update
  if (info == 10) return 0; // Skip
  const uint32_t lc = cp_clock(D, cp_cl_find(D, client));
  if (clock > lc) { // a gap: pending (not on the device)
    cp_unsup(D, CU_GAP);
    return -1;
  }
  Cur r{D.up, 0xFFFFFFFFu, bpos + 1u}; // validated by walk_update
  bool cn;
  uint32_t fl = 0, oc = 0, ok = 0, rc = 0, rk = 0;
  if (info != 0) {
    if (info & 0x80) {
      rd_var_u32(r, oc, cn);
      rd_var_u32(r, ok, cn);
      fl |= F_ORIGIN;
    }
    if (info & 0x40) {
      rd_var_u32(r, rc, cn);
      rd_var_u32(r, rk, cn);
      fl |= F_RO;
    }
    // Update::missing (update.rs:310-345)
    if ((fl & F_ORIGIN) && oc != client && ok >= cp_clock(D, cp_cl_find(D, oc))) {
      dep = oc;
      return 1;
    }
    if ((fl & F_RO) && rc != client && rk >= cp_clock(D, cp_cl_find(D, rc))) {
      dep = rc;
      return 1;
    }
  }
  // parent info (decode_block, update.rs:444-470): named root, ID of a type item, or from the
  // neighbours (origins present); parent_sub only with a written parent
  uint32_t pkind = 2, pc = 0, pk = 0, pno = 0, pnl = 0, pso = 0, psl = 0; // 0 named, 1 ID, 2 unknown
  if (info != 0 && (info & 0xC0) == 0) {
    uint32_t pi;
    rd_var_u32(r, pi, cn);
    if (pi == 1) {
      pkind = 0;
      rd_var_u32(r, pnl, cn);
      pno = r.i;
      r.i += pnl;
    } else {
      pkind = 1;
      rd_var_u32(r, pc, cn);
      rd_var_u32(r, pk, cn);
      if (pc != client && pk >= cp_clock(D, cp_cl_find(D, pc))) { // (Update::missing: the parent)
        dep = pc;
        return 1;
      }
    }
    if (info & 0x20) {
      rd_var_u32(r, psl, cn);
      pso = D.uoff + r.i;
      psl |= PS_HAS;
      r.i += psl & PS_LEN;
    }
  }
  const uint32_t offset = lc - clock;
  if (!(offset == 0 || offset < len)) return 0; // already known
  if (offset > 0) { // partially known: Item::integrate with an offset (not on the device)
    cp_unsup(D, CU_PARTIAL);
    return -1;
  }
  const int c = cp_cl_add(D, client);
  if (c < 0) return -1;
  const uint32_t x = cp_new_item(D);
  if (x == CNIL) return -1;
  D.I(x, I_CLOCK) = clock;
  D.I(x, I_LEN) = len;
  if (info == 0) { // GC
    D.I(x, I_FLAGS) = F_GC | ((uint32_t)c << 24);
    cp_push(D, c, x);
    return D.st ? -1 : 0;
  }
  fl |= (uint32_t)c << 24;
  D.I(x, I_OC) = oc;
  D.I(x, I_OK) = ok;
  D.I(x, I_RC) = rc;
  D.I(x, I_RK) = rk;
  D.I(x, I_PSO) = pso;
  D.I(x, I_PSL) = psl;
  // content (ItemContent::decode, block.rs:1786-1835)
  const uint32_t ref = info & 15;
  fl |= ref << 12;
  if (ref == 1) {
    fl |= F_DELC;
  } else if (ref == 4) { // String: one segment over the update's bytes
    uint32_t sl;
    rd_var_u32(r, sl, cn);
    const uint32_t s = cp_new_seg(D, D.uoff + r.i, sl | (sl == len ? SEG_ASCII : 0u));
    if (s == CNIL) return -1;
    D.I(x, I_SEG0) = D.I(x, I_SEG1) = s;
  } else if (ref == 8 || ref == 2) { // Any / JSON: one run of `len` elements
    uint32_t n;
    rd_var_u32(r, n, cn);
    if (ref == 2) n++; // (JSON: the count is len - 1)
    const uint32_t s = cp_new_seg(D, D.uoff + r.i, n);
    if (s == CNIL) return -1;
    D.I(x, I_SEG0) = D.I(x, I_SEG1) = s;
  } else { // Binary (buf) / Embed (json) / Format (key, json) / Type (type ref, name)
    const uint32_t c0 = r.i;
    uint32_t v;
    if (ref == 7) {
      const uint8_t tr = D.up[r.i++];
      if (tr == 7) { // WeakLink: not on the device
        cp_unsup(D, CU_UPDATE_SHAPE);
        return -1;
      }
      if (tr == 3) {
        rd_var_u32(r, v, cn);
        r.i += v;
      }
    } else {
      if (ref == 6) {
        rd_var_u32(r, v, cn);
        r.i += v;
      }
      rd_var_u32(r, v, cn);
      r.i += v;
    }
    const uint32_t sg = cp_new_seg(D, D.uoff + c0, r.i - c0);
    if (sg == CNIL) return -1;
    D.I(x, I_SEG0) = sg;
    D.I(x, I_SEG1) = CNIL; // (a Type: its branch, set by cp_integrate)
    fl |= F_OPQ;
  }
  D.I(x, I_FLAGS) = fl;
  // Item::repair (block.rs:1287-1350)
  if (fl & F_ORIGIN) D.I(x, I_LEFT) = cp_clean_end(D, D.I(x, I_OC), D.I(x, I_OK));
  if (fl & F_RO) D.I(x, I_RIGHT) = cp_clean_start(D, D.I(x, I_RC), D.I(x, I_RK));
  if (D.st) return -1;
  uint32_t par = CNIL;
  if (pkind == 0) { // Store::get_or_create_type
    for (uint32_t q = 0; q < D.nroot && par == CNIL; q++)
      if (D.m[M_ROOTLEN + q] == pnl && bytes_eq(D.p + D.m[M_ROOTOFF + q], D.up + pno, pnl)) par = D.m[M_ROOTBR + q];
    if (par == CNIL) {
      if (D.nroot == CP_MAXROOT) {
        cp_unsup(D, CU_ROOTS);
        return -1;
      }
      const uint32_t q = D.nroot++;
      par = cp_new_branch(D, CNIL, q);
      if (par == CNIL) return -1;
      D.m[M_ROOTOFF + q] = D.uoff + pno;
      D.m[M_ROOTLEN + q] = pnl;
      D.m[M_ROOTBR + q] = par;
    }
  } else if (pkind == 1) { // the type item's branch; Deleted content or not found: unknown
    const uint32_t pi = cp_get_item(D, pc, pk);
    if (pi != CNIL) {
      const uint32_t pf = D.I(pi, I_FLAGS);
      if (cp_ref(pf) == 7 && !(pf & F_DELC)) par = D.I(pi, I_SEG1);
      else if (!(pf & F_DELC)) { // "parent points to a block which is not a shared type"
        D.st = E_PANIC;
        return -1;
      }
    }
  } else { // TypePtr::Unknown: the parent (and parent_sub) of a neighbour
    const uint32_t l = D.I(x, I_LEFT), rt = D.I(x, I_RIGHT);
    const uint32_t src = (l != CNIL && D.I(l, I_PAR) != CNIL) ? l : (rt != CNIL && D.I(rt, I_PAR) != CNIL) ? rt : CNIL;
    if (src != CNIL) {
      par = D.I(src, I_PAR);
      D.I(x, I_PSO) = D.I(src, I_PSO);
      D.I(x, I_PSL) = D.I(src, I_PSL);
    }
  }
  if (par == CNIL) { // parent unknown: integrated as a GC struct (update.rs:239-243)
    D.I(x, I_FLAGS) = F_GC | ((uint32_t)c << 24);
    D.I(x, I_SEG0) = D.I(x, I_SEG1) = CNIL;
    cp_push(D, c, x);
    return D.st ? -1 : 0;
  }
  D.I(x, I_PAR) = par;
  const bool del = cp_integrate(D, x);
  cp_push(D, c, x);
  if (del && !D.st) cp_delete(D, x);
  return D.st ? -1 : 0;
}

// apply_delete (transaction.rs:472-578) of the update's DeleteSet in its table order
__device__ void cp_apply_delete(CDoc &D, uint32_t nent) {
  // HashMap::insert order of the entries (IdSet::decode) -> iteration positions
  uint32_t pos[16];
  ds_small_order(D.m + M_UE, nent, pos);
  uint32_t first[16];
  for (uint32_t e = 0, acc = 0; e < nent; e++) {
    first[e] = acc;
    acc += D.m[M_UEN + e];
  }
  for (uint32_t k = 0; k < nent && !D.st; k++) {
    uint32_t e = 0;
    while (e < nent && pos[e] != k) e++;
    if (e == nent) continue;
    const int c = cp_cl_find(D, D.m[M_UE + e]);
    if (c < 0) continue; // a client without blocks: dropped by yrs (transaction.rs:474-476)
    const uint32_t state = cp_clock(D, c);
    for (uint32_t q = 0; q < D.m[M_UEN + e] && !D.st; q++) {
      const uint32_t *rg = D.ur + 3 * (first[e] + q);
      const uint32_t clock = rg[1], clock_end = rg[2];
      if (clock >= state || state < clock_end) { // unapplied: pending delete set (not on the device)
        cp_unsup(D, CU_PENDING_DS);
        return;
      }
      uint32_t x = cp_cell(D, c, clock);
      if (x == CNIL || (D.I(x, I_FLAGS) & F_GC)) continue;
      if (!(D.I(x, I_FLAGS) & F_DEL) && D.I(x, I_CLOCK) < clock) {
        const uint32_t sp = cp_split(D, x, clock - D.I(x, I_CLOCK));
        if (sp != CNIL) {
          cp_merge_block(D, c, D.I(sp, I_CLOCK));
          x = sp;
        }
      }
      for (; x != CNIL && !D.st; x = D.I(x, I_CNEXT)) {
        if (D.I(x, I_FLAGS) & F_GC) continue;
        if (D.I(x, I_CLOCK) >= clock_end) break;
        if (D.I(x, I_FLAGS) & F_DEL) continue;
        if (D.I(x, I_CLOCK) + D.I(x, I_LEN) > clock_end) {
          const uint32_t sp = cp_split(D, x, clock_end - D.I(x, I_CLOCK));
          if (sp != CNIL) cp_merge_block(D, c, D.I(sp, I_CLOCK));
        }
        cp_delete(D, x);
      }
    }
  }
}

// ------------------------------------------------------------------ encode (store.rs:204-232)
// Output writer bounded by the document's slot; string bytes move 16 at a time (the loads of a
// group issue together instead of one load-store round trip per byte)
struct CpWriter {
  uint8_t *p;
  uint64_t n, cap;
  __device__ __forceinline__ void u8(uint8_t b) {
    if (n < cap) p[n] = b;
    n++;
  }
  __device__ void bytes(const uint8_t *s, uint32_t k) {
    if (n + k > cap) {
      n += k;
      return;
    }
    uint8_t *d = p + n;
    uint32_t i = 0;
    for (; i + 16 <= k; i += 16) {
      uint8_t t[16];
#pragma unroll
      for (int j = 0; j < 16; j++) t[j] = s[i + j];
#pragma unroll
      for (int j = 0; j < 16; j++) d[i + j] = t[j];
    }
    for (; i < k; i++) d[i] = s[i];
    n += k;
  }
};
// cp_encode's writer: the bytes gather in the lane's LDS stage (free after the update loop)
// and go to the slot CP_STAGE at a time.  Written straight to HBM, every item-word load after
// a byte store waited for the stores to complete (one counter covers loads and stores):
// encode was 29 % of k_compact on C2.  Bytes past `cap` are counted, not written.
struct CpBufWriter {
  uint8_t *p;      // the document's slot
  uint64_t n, cap; // bytes so far (flushed + buffered), slot capacity
  uint8_t *buf;    // CP_STAGE bytes of LDS
  uint32_t bn;     // buffered
  uint64_t fl;     // flushed (n == fl + bn)
  __device__ void put(const uint8_t *s, uint32_t k) { // k bytes to p + fl, bounded by cap
    const uint64_t lim = fl >= cap ? 0 : (fl + k <= cap ? k : cap - fl);
    uint8_t *d = p + fl;
    uint32_t i = 0;
    for (; i + 16 <= lim; i += 16) {
      uint8_t t[16];
#pragma unroll
      for (int j = 0; j < 16; j++) t[j] = s[i + j];
#pragma unroll
      for (int j = 0; j < 16; j++) d[i + j] = t[j];
    }
    for (; i < lim; i++) d[i] = s[i];
    fl += k;
  }
  __device__ void flush() {
    put(buf, bn);
    bn = 0;
  }
  __device__ __forceinline__ void u8(uint8_t b) {
    if (bn == CP_STAGE) flush();
    buf[bn++] = b;
    n++;
  }
  __device__ void bytes(const uint8_t *s, uint32_t k) {
    n += k;
    if (bn + k <= CP_STAGE) {
      for (uint32_t i = 0; i < k; i++) buf[bn + i] = s[i];
      bn += k;
      return;
    }
    flush();
    put(s, k);
  }
};
// ItemContent::encode of Binary / Embed / Format (block.rs:1731-1785; encoder.rs:170-179): the
// buffer and the key as they are (canonical length varints), the JSON values re-serialised
// (serde_json::from_str then Any::to_json: json_canon, already validated by the decode)
template <class W> __device__ void cp_opaque(const uint8_t *p, uint32_t ref, W &w) {
  Cur c{p, 0xFFFFFFFFu, 0};
  bool cn;
  uint32_t v;
  if (ref == 7) { // TypeRef::encode: the type ref, XmlElement's name
    const uint8_t tr = p[0];
    w.u8(tr);
    if (tr == 3) {
      c.i = 1;
      rd_var_u32(c, v, cn);
      w_str(w, p + c.i, v);
    }
    return;
  }
  if (ref == 6) {
    rd_var_u32(c, v, cn);
    w_str(w, p + c.i, v);
    c.i += v;
  }
  rd_var_u32(c, v, cn);
  if (ref == 3) {
    w_str(w, p + c.i, v);
    return;
  }
  Counter cnt;
  json_canon(p + c.i, v, cnt);
  w_var(w, cnt.n);
  json_canon(p + c.i, v, w);
}
template <class W> __device__ void cp_encode(CDoc &D, W &w) {
  // clients with blocks, descending
  uint32_t ord[CP_MAXCL], n = 0;
  for (uint32_t c = 0; c < D.ncl; c++)
    if (D.m[M_HEAD + c] != CNIL) {
      uint32_t j = n++;
      while (j > 0 && D.m[M_CLID + ord[j - 1]] < D.m[M_CLID + c]) {
        ord[j] = ord[j - 1];
        j--;
      }
      ord[j] = c;
    }
  w_var(w, n);
  for (uint32_t k = 0; k < n; k++) {
    const uint32_t c = ord[k];
    uint32_t cnt = 0;
    for (uint32_t x = D.m[M_HEAD + c]; x != CNIL; x = D.I(x, I_CNEXT)) cnt++;
    w_var(w, cnt);
    w_var(w, D.m[M_CLID + c]);
    w_var(w, D.I(D.m[M_HEAD + c], I_CLOCK));
    for (uint32_t x = D.m[M_HEAD + c]; x != CNIL; x = D.I(x, I_CNEXT)) {
      const uint32_t fl = D.I(x, I_FLAGS);
      if (fl & F_GC) {
        w.u8(0);
        w_var(w, D.I(x, I_LEN));
        continue;
      }
      // Item::encode (block.rs:1363-1369 info, slice.rs:199-251 with no offset)
      const uint32_t ref = (fl & F_DELC) ? 1 : cp_ref(fl);
      const uint32_t psl = D.I(x, I_PSL);
      w.u8((uint8_t)(((fl & F_ORIGIN) ? 0x80 : 0) | ((fl & F_RO) ? 0x40 : 0) | ((psl & PS_HAS) ? 0x20 : 0) | ref));
      if (fl & F_ORIGIN) {
        w_var(w, D.I(x, I_OC));
        w_var(w, D.I(x, I_OK));
      }
      if (fl & F_RO) {
        w_var(w, D.I(x, I_RC));
        w_var(w, D.I(x, I_RK));
      }
      if (!(fl & (F_ORIGIN | F_RO))) { // parent: a root's name, or the ID of a nested type's item
        const uint32_t b = D.I(x, I_PAR), bi = cp_bw(D, b, B_ITEM);
        if (bi == CNIL) {
          const uint32_t q = cp_bw(D, b, B_ROOT);
          w_var(w, 1);
          w_str(w, D.p + D.m[M_ROOTOFF + q], D.m[M_ROOTLEN + q]);
        } else {
          w_var(w, 0);
          w_var(w, D.m[M_CLID + D.cl_of(bi)]);
          w_var(w, D.I(bi, I_CLOCK));
        }
        if (psl & PS_HAS) w_str(w, D.p + D.I(x, I_PSO), psl & PS_LEN);
      }
      if (fl & F_DELC) {
        w_var(w, D.I(x, I_LEN));
      } else if (fl & F_OPQ) {
        const uint32_t sg = D.I(x, I_SEG0);
        cp_opaque(D.p + D.sg[3 * sg], ref, w);
      } else if (ref == 8 || ref == 2) { // element runs: Any values re-encoded, JSON strings as they are
        w_var(w, D.I(x, I_LEN)); // (JSON too: the decoder reads count + 1 texts, the encoder writes the count)
        for (uint32_t s = D.I(x, I_SEG0); s != CNIL; s = D.sg[3 * s + 2]) {
          Cur c{D.p, 0xFFFFFFFFu, D.sg[3 * s]};
          for (uint32_t q = 0; q < D.sg[3 * s + 1]; q++) {
            if (ref == 8) {
              bool re;
              any_walk(c, w, re);
            } else {
              uint32_t v;
              bool cn;
              rd_var_u32(c, v, cn);
              w_str(w, D.p + c.i, v);
              c.i += v;
            }
          }
        }
      } else {
        uint32_t tb = 0;
        for (uint32_t s = D.I(x, I_SEG0); s != CNIL; s = D.sg[3 * s + 2]) tb += D.sg[3 * s + 1] & SEG_LEN;
        w_var(w, tb);
        for (uint32_t s = D.I(x, I_SEG0); s != CNIL; s = D.sg[3 * s + 2])
          w.bytes(D.p + D.sg[3 * s], D.sg[3 * s + 1] & SEG_LEN);
      }
    }
  }
  // DeleteSet::from(&BlockStore): store clients in hashbrown order (entry per first push),
  // deleted blocks joined (IdRange::push), inserted into a new table (HashMap::insert)
  SmallHB<32> st, ds;
  st.init_empty();
  ds.init_empty();
  bool ex;
  for (uint32_t c = 0; c < D.ncl; c++) st.entry(D.m[M_CLID + c], c, ex);
  uint32_t nds = 0;
  for (uint32_t s = 0; s < st.buckets; s++) {
    if (!st.slot[s]) continue;
    const uint32_t c = st.slot[s] - 1;
    bool any = false;
    for (uint32_t x = D.m[M_HEAD + c]; x != CNIL && !any; x = D.I(x, I_CNEXT))
      any = D.I(x, I_FLAGS) & (F_GC | F_DEL);
    if (any) ds.insert(D.m[M_CLID + c], c, ex), nds++;
  }
  w_var(w, nds);
  for (uint32_t s = 0; s < ds.buckets; s++) {
    if (!ds.slot[s]) continue;
    const uint32_t c = ds.slot[s] - 1;
    // ranges: runs of deleted / GC blocks (adjacent ones join)
    uint32_t nr = 0;
    bool in = false;
    for (uint32_t x = D.m[M_HEAD + c]; x != CNIL; x = D.I(x, I_CNEXT)) {
      const bool del = D.I(x, I_FLAGS) & (F_GC | F_DEL);
      if (del && !in) nr++;
      in = del;
    }
    w_var(w, D.m[M_CLID + c]);
    w_var(w, nr);
    uint32_t rs = 0, re = 0;
    in = false;
    for (uint32_t x = D.m[M_HEAD + c];; x = D.I(x, I_CNEXT)) {
      const bool del = x != CNIL && (D.I(x, I_FLAGS) & (F_GC | F_DEL));
      if (del) {
        if (!in) rs = D.I(x, I_CLOCK);
        re = D.I(x, I_CLOCK) + D.I(x, I_LEN);
      } else if (in) {
        w_var(w, rs);
        w_var(w, re - rs);
      }
      in = del;
      if (x == CNIL) break;
    }
  }
}

// ------------------------------------------------------------------ the kernel
// the update at byte a (ulen bytes) copied into this lane's LDS stage as aligned dwords (the
// loads of a group issue together); the global bytes when it does not fit or there is no stage
__device__ const uint8_t *cp_stage(const uint8_t *bytes, uint64_t a, uint32_t ulen, uint8_t *stage) {
  if (!stage || ulen + 4 > CP_STAGE) return bytes + a;
  const uint64_t a4 = a & ~3ull;
  const uint32_t *src = (const uint32_t *)(bytes + a4), nd = (uint32_t)((a - a4) + ulen + 3) >> 2;
  uint32_t *dst = (uint32_t *)stage;
  for (uint32_t k = 0; k < nd; k += 8) {
    uint32_t t[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) t[j] = k + j < nd ? src[k + j] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 8; j++)
      if (k + j < nd) dst[k + j] = t[j];
  }
  return stage + (a - a4);
}

// document d of the batch (the kernel's lane body; tools/hostemu runs it on the CPU too)
__device__ void compact_doc(const BatchIn &b, const FastOut &o, uint32_t *hdr, const uint64_t *scr_off,
                            uint32_t *scr, uint32_t d, uint8_t *stage, uint32_t *misc) {
  uint64_t u0 = b.doc_upd[d], u1 = b.doc_upd[d + 1];
  const uint64_t B0 = b.upd_off[u0], B1 = b.upd_off[u1];
  const uint64_t slot = 2 * B0 + 64ull * d, cap = 2 * (B1 - B0) + 64;
  CDoc D;
  D.p = b.bytes + B0;
  uint32_t *h = hdr + (size_t)CP_HDR * d;
  D.h = h;
  D.ni = D.ns = D.ncl = D.nroot = 0;
  D.gen_i = D.gen_c = 0;
  D.st = 0;
  D.why = 0;
  int status = 0;
  // diagnostic (env YMERGE_STAMPS): s_memtime sums per phase -> o.stamps[16 d + k]:
  // 0 decode, 1 integrate, 2 apply_delete, 3 commit, 4 encode, 5 updates
  uint64_t tph[6] = {0, 0, 0, 0, 0, 0}, tq = o.stamps ? __builtin_amdgcn_s_memtime() : 0;
  auto lap = [&](int k) {
    if (o.stamps) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      tph[k] += now - tq;
      tq = now;
    }
  };
  if (h[H_OVER]) { // more than CP_MAXCL block clients / document bytes over 2^31
    status = E_UNSUPPORTED;
    D.why = h[H_OVER];
    u1 = u0;
  }
  // layout (cp_words): misc, items, segments, arrival arrays, update buffers (none when
  // the counts already put the document outside the device shape: the loop below is skipped)
  uint32_t *base = scr + scr_off[d];
  D.cap_i = D.cap_s = 3 * h[H_NB] + 2 * h[H_NR] + 64;
  D.mB = h[H_MB];
  D.mR = h[H_MR];
  D.m = misc ? misc : base; // the client table etc. in the lane's LDS words when given
  D.it = base + 1024;
  D.sg = D.it + (size_t)D.cap_i * I_W;
  D.cb = D.sg + (size_t)D.cap_s * 3;
  {
    uint32_t acc = 0; // arrival array offsets (pairs) after the counts
    const uint32_t hn = h[H_NCL];
    D.m[M_HNCL] = hn;
    for (uint32_t k = 0; k < hn; k++) {
      D.m[M_HCL + k] = h[H_CL + k];
      D.m[M_HCN + k] = h[H_CN + k];
      D.m[M_HCO + k] = acc;
      acc += h[H_CN + k];
    }
    D.ubr = D.cb + 2ull * (acc + 8);
  }
  D.ub = D.ubr + 4ull * D.mB;
  D.stk = D.ub + 4ull * D.mB;
  D.ur = D.stk + D.mB;
  D.mb = D.ur + 3ull * D.mR;
  D.tx = D.mb + 4ull * D.mR + 4;
  D.bt = D.tx + 3ull * D.cap_i;
  D.cap_b = h[H_NB] + CP_MAXROOT + 8;
  D.me = D.bt + (size_t)BR_W * D.cap_b;
  D.wk = D.me + (size_t)ME_W * D.cap_i;
  D.gm = D.wk + D.cap_i;
  D.nbr = D.nme = D.ngm = 0;
  for (uint64_t u = u0; u < u1 && !status; u++) {
    // transaction begin: clocks before it
    for (uint32_t c = 0; c < D.ncl; c++) D.m[M_BEFORE + c] = cp_clock(D, (int)c);
    D.nub = D.nur = D.nt = D.nm = 0;
    const uint64_t a = b.upd_off[u], z = b.upd_off[u + 1];
    const uint32_t ulen = (uint32_t)(z - a);
    D.uoff = (uint32_t)(a - B0);
    D.up = cp_stage(b.bytes, a, ulen, stage);
    CpSink sk{&D, D.up, 0, 0, 0, false};
    const int e = walk_update(D.up, ulen, sk);
    if (e) {
      status = e;
      break;
    }
    if (sk.over) {
      status = E_UNSUPPORTED, D.why = CU_UPDATE_SHAPE;
      break;
    }
    lap(0);
    tph[5]++;
    // Update::integrate order (update.rs:169-262): per-client queues by client descending
    // (a client's sections keep their stream order), blocks in order; a block whose
    // dependency on another client is missing waits on a stack while that client's queue runs
    uint32_t qc[CP_MAXCL], qh[CP_MAXCL], qe[CP_MAXCL], nq = 0;
    for (uint32_t i = 0; i < D.nub; i++) {
      const uint32_t cl = D.ubr[4 * i];
      uint32_t q = 0;
      while (q < nq && qc[q] != cl) q++;
      if (q == nq) {
        if (nq == CP_MAXCL) break;
        qc[nq] = cl;
        qe[nq++] = 0;
      }
      qe[q]++;
    }
    if (nq == CP_MAXCL && D.nub) { // (one more client cannot pass k_compact_count)
      uint32_t tot = 0;
      for (uint32_t q = 0; q < nq; q++) tot += qe[q];
      if (tot != D.nub) {
        status = E_UNSUPPORTED, D.why = CU_CLIENTS;
        break;
      }
    }
    for (uint32_t i = 1; i < nq; i++) { // clients descending
      const uint32_t c0 = qc[i], n0 = qe[i];
      uint32_t j = i;
      while (j > 0 && qc[j - 1] < c0) {
        qc[j] = qc[j - 1];
        qe[j] = qe[j - 1];
        j--;
      }
      qc[j] = c0;
      qe[j] = n0;
    }
    for (uint32_t q = 0, acc = 0; q < nq; q++) {
      qh[q] = acc;
      acc += qe[q];
      qe[q] = qh[q];
    }
    for (uint32_t i = 0; i < D.nub; i++) { // stable scatter; positions made document-relative
      uint32_t q = 0;
      while (qc[q] != D.ubr[4 * i]) q++;
      uint32_t *t = D.ub + 4 * qe[q]++;
      t[0] = D.ubr[4 * i];
      t[1] = D.ubr[4 * i + 1];
      t[2] = D.ubr[4 * i + 2];
      t[3] = D.ubr[4 * i + 3];
    }
    if (D.nub) {
      uint32_t sp = 0, cur = 0, head = qh[0]++;
      for (;;) {
        uint32_t dep = 0;
        const int rv = cp_block(D, D.ub + 4 * head, dep);
        if (rv < 0) break;
        if (rv == 1) {
          uint32_t q = 0;
          while (q < nq && qc[q] != dep) q++;
          if (sp == D.mB || q == nq || qh[q] == qe[q]) { // pending (not on the device)
            cp_unsup(D, CU_PENDING);
            break;
          }
          D.stk[sp++] = head;
          head = qh[q]++;
          continue;
        }
        if (sp) head = D.stk[--sp];
        else if (qh[cur] < qe[cur]) head = qh[cur]++;
        else {
          while (++cur < nq && qh[cur] == qe[cur]) {
          }
          if (cur == nq) break;
          head = qh[cur]++;
        }
      }
    }
    lap(1);
    if (!D.st) cp_apply_delete(D, sk.nent);
    lap(2);
    if (!D.st) cp_commit(D);
    lap(3);
    status = D.st;
  }
  uint64_t olen = 0;
  if (!status) { // one pass into the slot, bounded by its capacity
    if (stage) {
      CpBufWriter w{o.out + slot, 0, cap, stage, 0, 0};
      cp_encode(D, w);
      w.flush();
      if (w.n > cap) status = E_UNSUPPORTED, D.why = CU_OUTPUT;
      olen = w.n;
    } else {
      CpWriter w{o.out + slot, 0, cap};
      cp_encode(D, w);
      if (w.n > cap) status = E_UNSUPPORTED, D.why = CU_OUTPUT;
      olen = w.n;
    }
  }
  lap(4);
  if (o.stamps)
    for (int k = 0; k < 6; k++) o.stamps[(size_t)d * 16 + k] = tph[k];
  o.status[d] = (uint8_t)status;
  if (o.path) o.path[d] = (uint8_t)(status == E_UNSUPPORTED ? D.why : 0);
  o.out_start[d] = slot;
  o.out_len[d] = status ? 0 : olen;
}

// lpw documents per wavefront (lanes >= lpw idle): fewer lanes per wave trade SIMD width for
// less divergence and more waves in flight on a latency-bound, branchy lane body
__global__ void __launch_bounds__(64) k_compact(BatchIn b, FastOut o, uint32_t *hdr, const uint64_t *scr_off,
                                                 uint32_t *scr, uint32_t lpw) {
  __shared__ __align__(16) uint8_t stage[CP_LANES * CP_STAGE];
  __shared__ uint32_t misc[CP_LANES * M_END];
  ym_set_grammar(0);
  const uint32_t d = blockIdx.x * lpw + threadIdx.x;
  if (threadIdx.x < lpw && d < b.n_docs)
    compact_doc(b, o, hdr, scr_off, scr, d, stage + threadIdx.x * CP_STAGE, misc + threadIdx.x * M_END);
}

// ------------------------------------------------------------------ counts (scratch sizing)
struct CpCountSink {
  uint32_t *h;
  uint32_t ub, ur;
  __device__ void on_section(uint32_t) {}
  __device__ int on_block(uint32_t client, uint32_t, const BlockInfo &, uint32_t, uint32_t) {
    uint32_t k = 0;
    while (k < h[H_NCL] && h[H_CL + k] != client) k++;
    if (k == h[H_NCL]) {
      if (k == CP_MAXCL) {
        h[H_OVER] = CU_CLIENTS;
        return E_UNSUPPORTED; // stops the walk
      }
      h[H_CL + k] = client;
      h[H_CN + k] = 0;
      h[H_NCL] = k + 1;
    }
    h[H_CN + k]++;
    h[H_NB]++;
    ub++;
    return 0;
  }
  __device__ int on_ds_begin(uint32_t) { return 0; }
  __device__ int on_ds_entry(uint32_t, uint32_t) { return 0; }
  __device__ void on_ds_range(uint32_t, uint32_t) {
    h[H_NR]++;
    ur++;
  }
  __device__ int on_ds_done() { return 0; }
};
// document d: its count header and scratch words
__device__ void compact_count_doc(const BatchIn &b, uint32_t *hdr, uint64_t *need, uint32_t d, uint8_t *stage) {
  uint32_t *h = hdr + (size_t)CP_HDR * d;
  for (uint32_t i = 0; i < CP_HDR; i++) h[i] = 0;
  const uint64_t u0 = b.doc_upd[d], u1 = b.doc_upd[d + 1];
  if (b.upd_off[u1] - b.upd_off[u0] >= (1ull << 31)) {
    h[H_OVER] = CU_ITEMS;
  } else {
    CpCountSink sk{h, 0, 0};
    for (uint64_t u = u0; u < u1; u++) {
      sk.ub = sk.ur = 0;
      const uint64_t a = b.upd_off[u], z = b.upd_off[u + 1];
      const int e = walk_update(cp_stage(b.bytes, a, (uint32_t)(z - a), stage), (uint32_t)(z - a), sk);
      if (sk.ub > h[H_MB]) h[H_MB] = sk.ub;
      if (sk.ur > h[H_MR]) h[H_MR] = sk.ur;
      if (e || h[H_OVER]) break;
    }
  }
  need[d] = h[H_OVER] ? 0 : cp_words(h);
}
__global__ void __launch_bounds__(64) k_compact_count(BatchIn b, uint32_t *hdr, uint64_t *need) {
  __shared__ __align__(16) uint8_t stage[64 * CP_STAGE];
  ym_set_grammar(0);
  const uint32_t d = blockIdx.x * 64 + threadIdx.x;
  if (d < b.n_docs) compact_count_doc(b, hdr, need, d, stage + threadIdx.x * CP_STAGE);
}

void launch_compact_count(const BatchIn &b, uint32_t *hdr, uint64_t *need, hipStream_t s) {
  if (!b.n_docs) return;
  hipLaunchKernelGGL(k_compact_count, dim3((b.n_docs + 63) / 64), dim3(64), 0, s, b, hdr, need);
}
void launch_compact(const BatchIn &b, const FastOut &o, uint32_t *hdr, const uint64_t *scr_off, uint32_t *scr,
                    uint32_t lpw, hipStream_t s) {
  if (!b.n_docs) return;
  if (lpw < 1 || lpw > CP_LANES) lpw = CP_LANES; // the LDS arrays hold CP_LANES documents
  hipLaunchKernelGGL(k_compact, dim3((b.n_docs + lpw - 1) / lpw), dim3(64), 0, s, b, o, hdr, scr_off, scr, lpw);
}

} // namespace ym
