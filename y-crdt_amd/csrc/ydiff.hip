// ydiff.hip — batched diff_updates_v1 and encode_state_vector_from_update_v1 on gfx950.
//
// Reference semantics:
//   diff_updates_v1                    yrs/src/alt.rs:73-81 -> StateVector::decode
//                                      (state_vector.rs:111-124), Update::decode_v1
//                                      (update.rs:714-749), Update::encode_diff (update.rs:490-535),
//                                      IdSet::encode (id_set.rs:401-410), IdRange::encode
//                                      (id_set.rs:256-266: squash a clone when !is_squashed)
//   encode_state_vector_from_update_v1 yrs/src/alt.rs:54-57 -> Update::state_vector
//                                      (update.rs:107-114; BlockRange::last_id +1 quirk,
//                                      block.rs:1150-1152), StateVector::encode (state_vector.rs:126-134)
//
// Two kernels per batch (one update per document):
//   k_plan  — one lane per document walks its update once through a register window
//             (ywin.h): validation in stream order, per-client state (remote clock, first
//             block past the remote clock, section byte ranges), DeleteSet table order
//             (hashbrown emulation, GHB), squash of unsquashed ranges; emits a short list of
//             output ops with their sizes.  The small-capacity pass runs over every document
//             with a fixed per-document scratch; documents that overflow it are re-planned in
//             a second pass whose scratch is sized from the document length.
//   k_exec  — one wavefront per document: wave prefix scan of the op sizes, header / re-encode
//             ops lane-parallel, verbatim byte ranges (most of the output) copied by all 64
//             lanes with coalesced accesses.
#include "ycodec.h"
#include "yseq.h"
#include "ywin.h"
#include "ywalk.h"
#include "ylds.h"
#include "ywave.h"
#include "ykernels.h"

namespace ym {

enum : uint32_t { OP_VARS = 1, OP_COPY = 2, OP_EMIT = 3, OP_WALK = 4, OP_DSQ = 5, OP_DSS = 6, OP_SLICE = 7 };
constexpr uint32_t OPW = 8;  // words per op: kind, size, p0..p4, out offset
constexpr uint32_t CLW = 16; // words per client entry ([12..14]: first-block op hint, k_plan_ring)
constexpr uint32_t SECW = 5; // words per section record
constexpr uint32_t DEW = 8;  // words per DeleteSet entry
constexpr uint32_t PLAN_OVF = 0xFFFF;

struct PlanLayout {
  uint32_t BC, BE;
  uint32_t ct_slot, ct_keys, ct_tmp, cl, sec, dt_slot, dt_keys, dt_tmp, de, sq, s2_slot, s2_keys, s2_tmp, s2_val,
      ops, words;
};
__host__ __device__ inline uint32_t buckets_for(uint64_t cap) {
  if (cap < 8) return cap < 4 ? 4 : 8;
  uint64_t adj = cap * 8 / 7, b = 1;
  while (b < adj) b <<= 1;
  return (uint32_t)b;
}
__host__ __device__ inline PlanLayout plan_layout(const PlanCaps &c) {
  PlanLayout L;
  uint32_t o = 2; // [0] n ops, [1] reserved
  auto take = [&](uint32_t w) {
    uint32_t r = o;
    o += (w + 1) & ~1u;
    return r;
  };
  L.BC = buckets_for(c.C);
  L.BE = buckets_for(c.E);
  L.ct_slot = take(L.BC);
  L.ct_keys = take(c.C);
  L.ct_tmp = take(L.BC > c.C ? L.BC : c.C);
  L.cl = take(CLW * c.C);
  L.sec = take(SECW * c.C);
  L.dt_slot = take(L.BE);
  L.dt_keys = take(c.E);
  L.dt_tmp = take(L.BE);
  L.de = take(DEW * c.E);
  L.sq = take(2 * c.R);
  L.s2_slot = take(L.BC);
  L.s2_keys = take(c.C);
  L.s2_tmp = take(L.BC);
  L.s2_val = take(c.C);
  L.ops = take(OPW * c.O);
  L.words = o;
  return L;
}
// capacities that can never overflow for a successfully decoded update of `len` bytes:
// a client section takes >= 3 bytes, a DeleteSet entry >= 2, a range >= 2.
__host__ __device__ inline PlanCaps big_caps(uint64_t len) {
  PlanCaps c;
  c.C = (uint32_t)(len / 3 + 2);
  c.E = (uint32_t)(len / 2 + 2);
  c.R = (uint32_t)(len / 2 + 2);
  c.O = 3 * c.C + 2 * c.E + 4;
  return c;
}
__host__ __device__ inline PlanCaps small_caps() { return PlanCaps{8, 8, 64, 3 * 8 + 2 * 8 + 4}; }
uint64_t plan_small_words() { return plan_layout(small_caps()).words; }
__host__ __device__ inline uint64_t plan_big_words(uint64_t len) { return plan_layout(big_caps(len)).words; }

// canonical size of a validated block re-encoded with ItemSlice offset `off`
__device__ __forceinline__ int block_size(const WCur &c, uint32_t pos, uint32_t blen, const BlockInfo &bi,
                                          uint32_t client, uint32_t clock, uint32_t off, uint32_t &sz) {
  if (bi.kind != BK_ITEM) {
    sz = off == 0 && !bi.reenc ? blen : 1 + varlen(bi.len - off);
    return 0;
  }
  if (off == 0 && !bi.reenc) {
    sz = blen;
    return bi.enc_panic ? E_PANIC : 0;
  }
  Counter cn;
  int e = emit_block(c.p, c.n, pos, client, clock, bi.len, off, cn);
  sz = (uint32_t)cn.n;
  return e;
}

// remote clock of `client` in an encoded state vector (last entry wins: HashMap::insert)
__device__ __forceinline__ uint32_t sv_lookup(const uint8_t *sv, uint32_t n, uint32_t client) {
  WCur s;
  wc_init(s, sv, n);
  bool cn;
  uint32_t len, clk, r = 0;
  uint64_t c;
  if (wc_var_u32(s, len, cn)) return 0;
  for (uint32_t i = 0; i < len; i++) {
    if (wc_var_u64(s, c, cn) || wc_var_u32(s, clk, cn)) return r;
    if (c == (uint64_t)client) r = clk;
  }
  return r;
}

struct OpW {
  uint32_t *ops;
  uint32_t n, cap;
  __device__ bool put(uint32_t kind, uint32_t size, uint32_t a = 0, uint32_t b = 0, uint32_t c = 0, uint32_t d = 0,
                      uint32_t e = 0) {
    if (n >= cap) return false;
    uint32_t *o = ops + (size_t)OPW * n++;
    o[0] = kind;
    o[1] = size;
    o[2] = a;
    o[3] = b;
    o[4] = c;
    o[5] = d;
    o[6] = e;
    o[7] = 0;
    return true;
  }
};
__device__ __forceinline__ uint32_t vars_size(uint32_t k, uint32_t a, uint32_t b, uint32_t c) {
  uint32_t s = varlen(a);
  if (k > 1) s += varlen(b);
  if (k > 2) s += varlen(c);
  return s;
}

// The output plan of a fully walked document (shared by plan_doc and the ring planner):
// ops for encode_diff (clients descending, DeleteSet in table order) or the state vector.
template <bool DIFF>
__device__ __noinline__ uint32_t plan_finish(uint32_t *scr, const PlanLayout &L, const PlanCaps &cap, GHB &ct,
                                             uint32_t nsec, GHB &dt, bool unsupported, uint32_t pending,
                                             uint64_t &out_size) {
  const uint32_t *cl = scr + L.cl, *sec = scr + L.sec, *de = scr + L.de;
  OpW ow{scr + L.ops, 0, cap.O};
  uint64_t total = 0;
  if (DIFF) {
    if (unsupported) return E_UNSUPPORTED;
    if (pending) return pending;
    // clients with content, descending (encode_diff sorts by client id)
    uint32_t *ord = scr + L.ct_tmp;
    uint32_t nf = 0;
    for (uint32_t e = 0; e < ct.items; e++)
      if (cl[CLW * e + 5]) {
        const uint32_t k = ct.keys[e];
        uint32_t j = nf++;
        while (j > 0 && ct.keys[ord[j - 1]] < k) {
          ord[j] = ord[j - 1];
          j--;
        }
        ord[j] = e;
      }
    if (!ow.put(OP_VARS, varlen(nf), 1, nf)) return PLAN_OVF;
    total += varlen(nf);
    for (uint32_t q = 0; q < nf; q++) {
      const uint32_t e = ord[q];
      const uint32_t *st = cl + CLW * e;
      const uint32_t client = ct.keys[e];
      const uint32_t hclock = st[7] + st[9];
      uint32_t hs = vars_size(3, st[10], client, hclock);
      if (!ow.put(OP_VARS, hs, 3, st[10], client, hclock)) return PLAN_OVF;
      // first block past the remote clock: verbatim (canonical, offset 0), an ASCII / Deleted
      // slice written by the hot executor (ring planner), or emit_block (cold executor)
      const bool okf = st[14] == 1   ? ow.put(OP_COPY, st[11], st[6])
                       : st[14] == 2 ? ow.put(OP_SLICE, st[11], client, st[7] + st[9] - 1, st[12], st[13], st[8] - st[9])
                                     : ow.put(OP_EMIT, st[11], st[6], st[7], st[8], st[9], client);
      if (!okf) return PLAN_OVF;
      total += hs + st[11];
      for (uint32_t s = 0; s < nsec; s++) {
        const uint32_t *sr = sec + SECW * s;
        if (sr[0] != e || sr[1] >= sr[2]) continue;
        bool ok = sr[3] ? ow.put(OP_COPY, sr[2] - sr[1], sr[1]) : ow.put(OP_WALK, sr[4], sr[1], sr[2], 0, 0, client);
        if (!ok) return PLAN_OVF;
        total += sr[3] ? sr[2] - sr[1] : sr[4];
      }
    }
    // DeleteSet in table order
    if (!ow.put(OP_VARS, varlen(dt.items), 1, dt.items)) return PLAN_OVF;
    total += varlen(dt.items);
    for (uint32_t s = 0; s < dt.buckets; s++) {
      if (!dt.slot[s]) continue;
      const uint32_t *r = de + DEW * (dt.slot[s] - 1);
      const uint32_t vs = varlen(r[0]);
      bool ok = ow.put(OP_VARS, vs, 1, r[0]);
      if (r[4] & 1) {
        ok = ok && ((r[4] & 2) ? ow.put(OP_COPY, r[2] - r[1], r[1]) : ow.put(OP_DSS, r[7] - vs, r[1], r[3]));
      } else {
        ok = ok && ow.put(OP_DSQ, r[7] - vs, r[5], r[6]);
      }
      if (!ok) return PLAN_OVF;
      total += r[7];
    }
  } else {
    // Update::state_vector: iterate the decoded client table, set_max into a fresh table
    GHB s2{scr + L.s2_slot, scr + L.s2_keys, L.BC, 0, 0, 0};
    uint32_t *val = scr + L.s2_val;
    for (uint32_t s = 0; s < ct.buckets; s++) {
      if (!ct.slot[s]) continue;
      const uint32_t e = ct.slot[s] - 1;
      const uint32_t *st = cl + CLW * e;
      if (st[0] == 0) return E_PANIC; // blocks[blocks.len() - 1] on an empty deque
      // last_id().clock + 1: Item -> clock + len; GC / Skip -> clock + len + 1 (block.rs:1150-1152)
      const uint32_t v = st[2] + st[3] + ((st[1] & 0xFF) != BK_ITEM ? 1u : 0u);
      const uint32_t key = ct.keys[e];
      int f = s2.find(key);
      if (f < 0) {
        f = (int)s2.items;
        if (!s2.reserve(1, scr + L.s2_tmp)) return PLAN_OVF;
        s2.place(key, (uint32_t)f);
        val[f] = 0;
      }
      if (v > val[f]) val[f] = v;
    }
    if (!ow.put(OP_VARS, varlen(s2.items), 1, s2.items)) return PLAN_OVF;
    total += varlen(s2.items);
    for (uint32_t s = 0; s < s2.buckets; s++) {
      if (!s2.slot[s]) continue;
      const uint32_t e = s2.slot[s] - 1;
      const uint32_t k = s2.keys[e], v = val[e];
      const uint32_t sz = varlen(k) + varlen(v);
      if (!ow.put(OP_VARS, sz, 2, k, v)) return PLAN_OVF;
      total += sz;
    }
  }
  scr[0] = ow.n;
  out_size = total;
  return 0;
}

// Plans one document.  Returns PLAN_OVF when the scratch capacities are exceeded (the
// document is re-planned with big capacities), otherwise the yrs status (0 = ok).
template <bool DIFF>
__device__ uint32_t plan_doc(const uint8_t *up, uint32_t un, const uint8_t *svp, uint32_t svn, uint32_t *scr,
                             const PlanCaps &cap, uint64_t &out_size) {
  const PlanLayout L = plan_layout(cap);
  bool cn;
  // ---- remote state vector (decoded before the update, alt.rs:77-78)
  if (DIFF) {
    WCur s;
    wc_init(s, svp, svn);
    uint32_t len, clk;
    uint64_t c;
    YM_TRY(wc_var_u32(s, len, cn));
    if (len && (uint64_t)buckets_for(len) * 17ull > ALLOC_LIMIT) return E_PANIC; // with_capacity
    for (uint32_t i = 0; i < len; i++) {
      YM_TRY(wc_var_u64(s, c, cn));
      YM_TRY(wc_var_u32(s, clk, cn));
    }
  }
  // ---- update: client sections
  WCur c;
  wc_init(c, up, un);
  uint32_t ncl;
  YM_TRY(wc_var_u32(c, ncl, cn));
  if (ncl && (uint64_t)buckets_for(ncl) * 41ull > ALLOC_LIMIT) return E_NEM; // try_reserve
  GHB ct{scr + L.ct_slot, scr + L.ct_keys, L.BC, 0, 0, 0};
  if (ncl && !ct.reserve(ncl, scr + L.ct_tmp)) return PLAN_OVF;
  uint32_t *cl = scr + L.cl, *sec = scr + L.sec;
  uint32_t nsec = 0;
  uint32_t pending = 0; // first encode-time error (yrs encodes only after a full decode)
  bool unsupported = false;
  for (uint32_t i = 0; i < ncl; i++) {
    uint32_t nb, client, clock;
    YM_TRY(wc_var_u32(c, nb, cn));
    YM_TRY(wc_var_u32(c, client, cn));
    YM_TRY(wc_var_u32(c, clock, cn));
    int e = ct.find(client);
    if (e < 0) { // entry(..).or_default: capacity reserved up front
      e = (int)ct.items;
      if (!ct.reserve(1, scr + L.ct_tmp)) return PLAN_OVF;
      ct.place(client, (uint32_t)e);
      uint32_t *s = cl + CLW * e;
      for (uint32_t k = 0; k < CLW; k++) s[k] = 0;
      if (DIFF) s[4] = sv_lookup(svp, svn, client);
    }
    uint32_t *st = cl + CLW * e;
    uint32_t nstored = st[0], lkind = st[1], lclock = st[2], llen = st[3];
    const uint32_t remote = st[4];
    uint32_t found = st[5], count = st[10];
    if (((uint64_t)nstored + nb) * 32ull > ALLOC_LIMIT) return E_NEM;
    if (nsec >= cap.C) return PLAN_OVF;
    uint32_t kb = 0xFFFFFFFFu, pure = 1, ssize = 0;
    for (uint32_t j = 0; j < nb; j++) {
      const uint32_t bpos = c.i;
      BlockInfo bi;
      YM_TRY(wparse_block(c, bi));
      if (bi.kind == BK_ITEM && bi.len == 0) { // Item::new -> None: dropped
        if (kb != 0xFFFFFFFFu) pure = 0;
        continue;
      }
      if ((uint64_t)clock + bi.len > 0xFFFFFFFFull) return E_PANIC;
      unsupported |= bi.unsupported;
      nstored++;
      lkind = bi.kind;
      lclock = clock;
      llen = bi.len;
      if (DIFF) {
        const uint32_t blen = c.i - bpos;
        if (!found) {
          if (bi.kind != BK_SKIP && clock + bi.len > remote) {
            found = 1;
            const uint32_t off = remote > clock ? remote - clock : 0;
            uint32_t sz = 0;
            if (!bi.unsupported) {
              int ee = block_size(c, bpos, blen, bi, client, clock, off, sz);
              if (ee && !pending) pending = (uint32_t)ee;
            }
            st[6] = bpos;
            st[7] = clock;
            st[8] = bi.len;
            st[9] = off;
            st[11] = sz;
            if (off == 0 && !bi.reenc && !bi.enc_panic && !bi.unsupported) st[14] = 1; // bytes as they are
            count = 1;
            kb = c.i;
          }
        } else {
          if (kb == 0xFFFFFFFFu) kb = bpos;
          count++;
          uint32_t sz = blen;
          if (bi.reenc || bi.enc_panic) {
            pure = 0;
            if (!bi.unsupported) {
              int ee = block_size(c, bpos, blen, bi, client, clock, 0, sz);
              if (ee && !pending) pending = (uint32_t)ee;
            }
          }
          ssize += sz;
        }
      }
      clock += bi.len;
    }
    if (kb == 0xFFFFFFFFu) kb = c.i;
    uint32_t *sr = sec + SECW * nsec++;
    sr[0] = (uint32_t)e;
    sr[1] = kb;
    sr[2] = c.i;
    sr[3] = pure;
    sr[4] = ssize;
    st[0] = nstored;
    st[1] = lkind | 0x100;
    st[2] = lclock;
    st[3] = llen;
    st[5] = found;
    st[10] = count;
  }
  // ---- DeleteSet (IdSet::decode: HashMap::insert per entry, id_set.rs:412-426)
  uint32_t nds;
  YM_TRY(wc_var_u32(c, nds, cn));
  GHB dt{scr + L.dt_slot, scr + L.dt_keys, L.BE, 0, 0, 0};
  uint32_t *de = scr + L.de, *sq = scr + L.sq;
  uint32_t nsq = 0;
  for (uint32_t i = 0; i < nds; i++) {
    uint32_t client, n;
    YM_TRY(wc_var_u32(c, client, cn));
    const uint32_t cpos = c.i;
    YM_TRY(wc_var_u32(c, n, cn));
    bool canon = cn, squashed = true;
    uint32_t prev_e = 0, sz = varlen(n);
    for (uint32_t k = 0; k < n; k++) {
      uint32_t s0, ln;
      wc_ensure(c, 20);
      YM_TRY(wc_var_u32(c, s0, cn));
      canon &= cn;
      YM_TRY(wc_var_u32(c, ln, cn));
      canon &= cn;
      if ((uint64_t)s0 + ln > 0xFFFFFFFFull) return E_PANIC;
      if (k > 0 && s0 < prev_e) squashed = false;
      prev_e = s0 + ln;
      sz += varlen(s0) + varlen(ln);
    }
    if (!DIFF) continue;
    if (i >= cap.E) return PLAN_OVF;
    if (!dt.reserve(1, scr + L.dt_tmp)) return PLAN_OVF;
    int e = dt.find(client);
    if (e >= 0) { // replaced in place: the slot now names entry i
      for (uint32_t s = 0; s < dt.buckets; s++)
        if (dt.slot[s] == (uint32_t)e + 1) dt.slot[s] = i + 1;
      dt.keys[i] = client;
    } else {
      dt.place(client, i);
    }
    uint32_t *r = de + DEW * i;
    r[0] = client;
    r[1] = cpos;
    r[2] = c.i;
    r[3] = n;
    r[4] = (squashed ? 1u : 0u) | (canon ? 2u : 0u);
    if (!squashed) {
      // IdRange::squash of a clone: stable sort by start, join overlapping or adjacent
      if (nsq + n > cap.R) return PLAN_OVF;
      uint32_t *v = sq + 2 * nsq;
      WCur q;
      wc_init(q, up, un);
      q.i = cpos;
      uint32_t dummy;
      wc_var_u32(q, dummy, cn);
      for (uint32_t k = 0; k < n; k++) {
        uint32_t s0, ln;
        wc_var_u32(q, s0, cn);
        wc_var_u32(q, ln, cn);
        // insertion into the sorted prefix (stable: after equal starts)
        uint32_t j = k;
        while (j > 0 && v[2 * (j - 1)] > s0) {
          v[2 * j] = v[2 * (j - 1)];
          v[2 * j + 1] = v[2 * (j - 1) + 1];
          j--;
        }
        v[2 * j] = s0;
        v[2 * j + 1] = s0 + ln;
      }
      uint32_t m = 0;
      for (uint32_t k = 0; k < n; k++) {
        uint32_t s0 = v[2 * k], e0 = v[2 * k + 1];
        if (m > 0 && !(v[2 * (m - 1)] > e0 || s0 > v[2 * (m - 1) + 1])) {
          if (s0 < v[2 * (m - 1)]) v[2 * (m - 1)] = s0;
          if (e0 > v[2 * (m - 1) + 1]) v[2 * (m - 1) + 1] = e0;
        } else {
          v[2 * m] = s0;
          v[2 * m + 1] = e0;
          m++;
        }
      }
      sz = varlen(m);
      for (uint32_t k = 0; k < m; k++) sz += varlen(v[2 * k]) + varlen(v[2 * k + 1] - v[2 * k]);
      r[5] = nsq;
      r[6] = m;
      nsq += m;
    }
    r[7] = varlen(client) + sz;
  }
  return plan_finish<DIFF>(scr, L, cap, ct, nsec, dt, unsupported, pending, out_size);
}

// Validation only (first error in stream order), for documents whose section count
// exceeds even the big capacities: such an update cannot decode (a section takes
// >= 3 bytes), so only its error code is needed.
struct NullSink {
  YM_INLINE void on_section(uint32_t) {}
  YM_INLINE int on_block(uint32_t, uint32_t, const BlockInfo &, uint32_t, uint32_t) { return 0; }
  YM_INLINE int on_ds_begin(uint32_t) { return 0; }
  YM_INLINE int on_ds_entry(uint32_t, uint32_t) { return 0; }
  YM_INLINE void on_ds_range(uint32_t, uint32_t) {}
  YM_INLINE int on_ds_done() { return 0; }
};
template <bool DIFF>
__device__ __noinline__ uint32_t validate_doc(const uint8_t *up, uint32_t un, const uint8_t *svp, uint32_t svn) {
  if (DIFF) {
    Cur s{svp, svn, 0};
    bool cn;
    uint32_t len, clk;
    uint64_t c;
    YM_TRY(rd_var_u32(s, len, cn));
    if (len && (uint64_t)buckets_for(len) * 17ull > ALLOC_LIMIT) return E_PANIC;
    for (uint32_t i = 0; i < len; i++) {
      YM_TRY(rd_var_u64(s, c, cn));
      YM_TRY(rd_var_u32(s, clk, cn));
    }
  }
  NullSink ns;
  int e = walk_update(up, un, ns);
  return e ? (uint32_t)e : (uint32_t)E_OTHER;
}

// ------------------------------------------------------------------ ring planner
// k_plan_ring: the common-shape planner.  Lane per document (a C5 batch has ~100k documents:
// one lane each is the instruction-cheapest walk), but each lane reads its update from a
// private 192-byte LDS ring instead of HBM: the ring is refilled with twelve 16-byte loads at
// one program point of the step loop, so a wave waits for memory once per refill round instead
// of once per block.  One step consumes one whole item — a block, a section header, a
// DeleteSet entry header or range — with branch-free LEB128 decodes of 8-byte LDS reads, so
// lanes of a wave stay converged on the item kind that dominates (string blocks).  Shapes it
// does not plan — a decode error, cold content kinds, non-ASCII strings, non-canonical blocks,
// unsquashed DeleteSet ranges, more than 8 clients / DeleteSet entries, a varint longer than 5
// bytes, a block header longer than the ring — leave the document to the general planner
// (k_plan pass 0), marked ps.big[d] = PLAN_REDO; everything it plans is byte-identical to it.
#ifndef YM_RING
#define YM_RING 192
#endif
constexpr uint32_t RING = YM_RING;      // ring bytes per lane (a multiple of 64)
constexpr uint32_t RING_STRIDE = RING + 16; // LDS bytes per lane (16-byte aligned rows)
constexpr uint32_t RING_G = RING % 128 == 0 ? 8 : 4; // 16-byte loads per refill group
constexpr uint32_t RING_NT = 256;       // lanes (documents) per workgroup
constexpr uint32_t RING_STEPS = 10;     // item steps between refill points
constexpr uint32_t LP_SLOW = 6;         // k_plan_lane: lanes that wait for a full step before the wave runs it
constexpr uint32_t LP_STEPS = 8;        // k_plan_lane: item steps between refill points (C5 sweep: 8 steps with
                                        // LP_SLOW 6 best, profiles/r04/r04n_lane_sweep.txt)
constexpr uint8_t PLAN_REDO = 3;
constexpr uint8_t PLAN_WAVE = 4;         // planned by k_plan_wave (k_plan_lane's long documents)
constexpr uint64_t PW_MIN = 64 * 1024;   // update bytes from which a document gets a wavefront

enum : uint32_t { R_NCL, R_SEC, R_BLOCK, R_NDS, R_DENT, R_DRANGE, R_DONE };

// 8 stream bytes at ring byte offset o (o + 8 <= RING_STRIDE): three dword reads + alignbyte
__device__ __forceinline__ uint64_t ring_read8(const uint32_t *row, uint32_t o) {
  const uint32_t w = o >> 2, sh = o & 3;
  const uint32_t d0 = row[w], d1 = row[w + 1], d2 = row[w + 2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh), hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Per-lane reader over the ring.  Every read checks that its 8 bytes are in the ring (else
// `fail` = F_SHORT: the step is retried after a refill) and that the value ends inside the
// stream (else F_BAIL, like any decode error or a varint longer than 5 bytes).
enum : uint32_t { F_OK = 0, F_SHORT = 1, F_BAIL = 2 };
struct RingRd {
  const uint32_t *row;
  uint64_t sbase, rb, rend, send;
  uint32_t un, fail;
  int32_t rbq, rendq; // the ring's start and end relative to the update (32-bit hot path)
  __device__ __forceinline__ void sync_rel() {
    rbq = (int32_t)(int64_t)(rb - sbase);
    rendq = (int32_t)(int64_t)(rend - sbase);
  }
  __device__ __forceinline__ uint64_t at(uint32_t q) {
    if (fail) return 0;
    if (q >= un) {
      fail = F_BAIL;
      return 0;
    }
    if ((int32_t)q + 8 > rendq && rendq != (int32_t)un) {
      fail = F_SHORT;
      return 0;
    }
    return ring_read8(row, (uint32_t)((int32_t)q - rbq));
  }
  // read_var_u32 (varint.rs:244-260, wrapping_shl) at q: bytes consumed; canon = the
  // re-encoding is the same bytes (no zero top group; a 5th byte below 16)
  __device__ __forceinline__ uint32_t var(uint32_t q, uint32_t &v, bool &canon) {
    const uint64_t x = at(q);
    const uint64_t m = ~x & 0x0000008080808080ull;
    uint32_t nb = ((uint32_t)__builtin_ctzll(m | (1ull << 63)) >> 3) + 1;
    if (!fail && (nb > 5 || nb > un - q)) fail = F_BAIL;
    if (fail) nb = 1;
    const uint64_t xm = x & (nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1));
    v = (uint32_t)((xm & 0x7F) | ((xm >> 1) & 0x3F80) | ((xm >> 2) & 0x1FC000) | ((xm >> 3) & 0xFE00000) |
                   ((xm >> 4) & 0x7F0000000ull));
    const uint32_t last = (uint32_t)(xm >> (8 * (nb - 1))) & 0xFF;
    canon = nb == 1 || (last != 0 && (nb < 5 || last < 16));
    return nb;
  }
};

template <bool DIFF>
__global__ void __launch_bounds__(RING_NT) k_plan_ring(DiffBatch b, PlanScratch ps) {
  ym_set_grammar(b.v1x);
  __shared__ __align__(16) uint32_t ring_lds[RING_NT * RING_STRIDE / 4];
  const uint32_t t = threadIdx.x;
  const uint32_t d = blockIdx.x * RING_NT + t;
  uint32_t *row = ring_lds + t * (RING_STRIDE / 4);
  bool active = d < b.n_docs;
  if (active && b.pre_status && b.pre_status[d]) { // e.g. a y-sync message that is not SyncStep1
    ps.big[d] = 0;
    ps.status[d] = b.pre_status[d];
    ps.size[d] = 0;
    active = false;
  }
  if (active && b.ls_done && b.ls_done[d]) active = false; // the long-update grid path's (ylong.hip)
  const uint8_t *up = nullptr, *svp = nullptr;
  uint32_t un = 0, svn = 0, nsv = 0;
  uint32_t *scr = nullptr;
  const PlanCaps cap = small_caps();
  const PlanLayout L = plan_layout(cap);
  bool bail = false;
  if (active) {
    const uint64_t o0 = b.upd_off[d], o1 = b.upd_off[d + 1];
    up = b.bytes + o0;
    un = (uint32_t)(o1 - o0);
    if (o1 - o0 >= (1ull << 31)) bail = true;
    scr = ps.small + (size_t)d * ps.small_words;
    if (DIFF && !bail) { // remote state vector, decoded before the update (alt.rs:77-78)
      svp = b.sv + b.sv_off[d];
      svn = (uint32_t)((b.sv_end ? b.sv_end[d] : b.sv_off[d + 1]) - b.sv_off[d]);
      // entries with a u32 client id go to a small table (the sq region: unsquashed ranges
      // are the general planner's); a client listed twice keeps its last clock (HashMap::insert)
      Cur s{svp, svn, 0};
      bool cn;
      uint32_t len = 0, clk;
      uint64_t c;
      if (rd_var_u32(s, len, cn) || (len && (uint64_t)buckets_for(len) * 17ull > ALLOC_LIMIT)) bail = true;
      uint32_t *svt = scr + L.sq;
      for (uint32_t i = 0; i < len && !bail; i++) {
        if (rd_var_u64(s, c, cn) || rd_var_u32(s, clk, cn)) {
          bail = true;
          break;
        }
        if (c >> 32) continue;
        uint32_t k = 0;
        while (k < nsv && svt[2 * k] != (uint32_t)c) k++;
        if (k == nsv) {
          if (nsv == cap.R / 2) {
            bail = true;
            break;
          }
          nsv++;
        }
        svt[2 * k] = (uint32_t)c;
        svt[2 * k + 1] = clk;
      }
    }
    if (bail) active = false;
  }
  GHB ct{scr + L.ct_slot, scr + L.ct_keys, L.BC, 0, 0, 0};
  GHB dt{scr + L.dt_slot, scr + L.dt_keys, L.BE, 0, 0, 0};
  uint32_t *cl = scr + L.cl, *sec = scr + L.sec, *de = scr + L.de;
  uint32_t st = R_NCL, pos = 0, ncl = 0, isec = 0, nb = 0, j = 0, client = 0, clock = 0, nclients = 0;
  // current section (plan_doc's per-client record, kept in registers while the section runs)
  uint32_t e = 0, nstored = 0, lkind = 0, lclock = 0, llen = 0, remote = 0, found = 0, count = 0, kb = 0, pure = 1,
           ssize = 0, nsec = 0;
  // DeleteSet
  uint32_t nds = 0, ids = 0, dclient = 0, cpos = 0, nr = 0, kr = 0, prev_e = 0, dsz = 0;
  bool dcanon = true, dsq = true;
  RingRd R{row, (uint64_t)up, 0, 0, (uint64_t)up + un, un, F_OK, 0, 0};
  bool have = false, wait = false;

  // diagnostic stamps (wave time): refill, steps, finish; refill rounds, step iterations
  uint64_t t_ref = 0, t_stp = 0, n_ref = 0, n_stp = 0, tq = ps.stamps ? __builtin_amdgcn_s_memtime() : 0;
  for (;;) {
    if (!__any(active)) break;
    if (ps.stamps) tq = __builtin_amdgcn_s_memtime();
    // ---- refill point: lanes that ran short, or are within 64 bytes of their ring's end
    const uint64_t a0 = R.sbase + pos;
    if (active && (!have || wait || (a0 + 64 > R.rb + RING && R.rb + RING < R.send))) {
      if (have && wait && R.rb == (a0 & ~15ull)) { // an item longer than a fresh ring
        bail = true;
        active = false;
      } else {
        R.rb = a0 & ~15ull;
        const uint4 *q = (const uint4 *)R.rb;
        uint4 *dst = (uint4 *)row;
#pragma unroll
        for (uint32_t g = 0; g < RING / 16; g += RING_G) { // groups of 16-byte loads
          uint4 x[RING_G];
#pragma unroll
          for (uint32_t k = 0; k < RING_G; k++)
            x[k] = R.rb + 16 * (g + k) < R.send ? q[g + k] : make_uint4(0, 0, 0, 0);
#pragma unroll
          for (uint32_t k = 0; k < RING_G; k++) dst[g + k] = x[k];
        }
        R.rend = R.rb + RING < R.send ? R.rb + RING : R.send;
        R.sync_rel();
        have = true;
        wait = false;
      }
    }
    if (ps.stamps) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      t_ref += now - tq;
      tq = now;
      n_ref++;
    }
    for (uint32_t step = 0; step < RING_STEPS; step++) {
      const bool can = active && !wait;
      if (!__any(can)) break;
      if (ps.stamps) n_stp++;
      if (!can) continue;
      R.fail = F_OK;
      bool cn, sec_end = false, entry_end = false;
      uint32_t q = pos, v;
      if (st == R_BLOCK) {
        // ---- one block (Update::decode_block, update.rs:433-488 + ItemContent::decode)
        const uint32_t info = (uint32_t)(R.at(q) & 0xFF);
        q++;
        bool reenc = false;
        uint32_t kind = BK_ITEM, len = 0, rbytes = 0, ropos = 0;
        if (info == 10 || info == 0) {
          kind = info == 10 ? BK_SKIP : BK_GC;
          q += R.var(q, len, cn);
          reenc = !cn;
        } else {
          uint32_t want = info & 0xCF; // 0x10 never re-emitted; 0x20 only when parent_sub decoded
          if (info & 0x80) {
            q += R.var(q, v, cn);
            reenc |= !cn;
            q += R.var(q, v, cn);
            reenc |= !cn;
          }
          ropos = q;
          if (info & 0x40) {
            uint32_t n1 = R.var(q, v, cn);
            reenc |= !cn;
            q += n1;
            uint32_t n2 = R.var(q, v, cn);
            reenc |= !cn;
            q += n2;
            rbytes = n1 + n2;
          }
          if ((info & 0xC0) == 0) {
            uint32_t pi;
            q += R.var(q, pi, cn);
            reenc |= !cn || pi > 1;
            if (pi == 1) {
              q += R.var(q, v, cn);
              reenc |= !cn;
              if (!R.fail && v > un - q) R.fail = F_BAIL;
              q += v;
            } else {
              q += R.var(q, v, cn);
              reenc |= !cn;
              q += R.var(q, v, cn);
              reenc |= !cn;
            }
            if (info & 0x20) {
              want |= 0x20;
              q += R.var(q, v, cn);
              reenc |= !cn;
              if (!R.fail && v > un - q) R.fail = F_BAIL;
              q += v;
            }
          }
          if (want != info) reenc = true;
          const uint32_t ref = info & 15;
          if (ref == 1) {
            q += R.var(q, len, cn);
            reenc |= !cn;
          } else if (ref == 4) {
            uint32_t slen;
            q += R.var(q, slen, cn);
            reenc |= !cn;
            if (!R.fail && slen > un - q) R.fail = F_BAIL;
            if (!R.fail && slen > 1) { // v == 1: one UTF-16 unit whatever the byte (wparse_block)
              uint64_t hib = 0;
              const uint64_t a = R.sbase + q;
              if (a + slen + 8 <= R.rend || (R.rend == R.send && a + slen <= R.rend)) {
                for (uint32_t k = 0; k < slen; k += 8) {
                  const uint32_t n8 = slen - k < 8 ? slen - k : 8;
                  hib |= ring_read8(row, (uint32_t)(a + k - R.rb)) & (n8 == 8 ? ~0ull : ((1ull << (8 * n8)) - 1));
                }
              } else { // payload past the ring: read it from HBM (the lane refills after it)
                for (uint32_t k = 0; k < slen; k++) hib |= up[q + k];
                wait = true;
              }
              if (hib & 0x8080808080808080ull) R.fail = F_BAIL; // non-ASCII: UTF-16 length / split checks
            }
            len = slen;
            q += slen;
          } else {
            R.fail = F_BAIL; // cold content kinds
          }
        }
        if (!R.fail && reenc) R.fail = F_BAIL; // re-encoded sizes: general planner
        if (!R.fail) {
          const uint32_t bpos = pos, blen = q - pos;
          pos = q;
          if (kind == BK_ITEM && len == 0) { // Item::new -> None: dropped
            if (kb != 0xFFFFFFFFu) pure = 0;
          } else if ((uint64_t)clock + len > 0xFFFFFFFFull) {
            R.fail = F_BAIL;
          } else {
            nstored++;
            lkind = kind;
            lclock = clock;
            llen = len;
            if (DIFF) {
              if (!found) {
                if (kind != BK_SKIP && clock + len > remote) {
                  found = 1;
                  const uint32_t off = remote > clock ? remote - clock : 0;
                  uint32_t sz;
                  if (off == 0) {
                    sz = blen;
                  } else if (kind != BK_ITEM) {
                    sz = 1 + varlen(len - off);
                  } else {
                    // ItemSlice::encode with an offset (emit_block): origin (client, clock + off - 1)
                    // synthesised, right origin copied (canonical here), no parent info, content
                    // sliced (ASCII string: byte offset = UTF-16 offset)
                    const uint32_t rest = len - off;
                    sz = 1 + varlen(client) + varlen(clock + off - 1) + rbytes + varlen(rest) +
                         ((info & 15) == 4 ? rest : 0u);
                  }
                  uint32_t *sr = cl + CLW * e;
                  sr[6] = bpos;
                  sr[7] = clock;
                  sr[8] = len;
                  sr[9] = off;
                  sr[11] = sz;
                  if (off == 0) {
                    sr[14] = 1;
                  } else if (kind == BK_ITEM) { // OP_SLICE: right origin bytes, ref, parent_sub flag
                    const uint32_t has_ps = (info & 0xE0) == 0x20 ? 1u : 0u;
                    sr[12] = ropos;
                    sr[13] = rbytes | ((info & 15) << 8) | (has_ps << 12) | ((pos - ropos) << 16);
                    sr[14] = 2;
                  }
                  count = 1;
                  kb = pos;
                }
              } else {
                if (kb == 0xFFFFFFFFu) kb = bpos;
                count++;
                ssize += blen;
              }
            }
            clock += len;
          }
          if (!R.fail && ++j == nb) sec_end = true;
        }
      } else if (st == R_SEC) {
        // ---- section header: blocks count, client, first clock
        q += R.var(q, nb, cn);
        q += R.var(q, client, cn);
        q += R.var(q, clock, cn);
        if (!R.fail) {
          pos = q;
          uint32_t f = 0;
          while (f < nclients && ct.keys[f] != client) f++;
          if (f == nclients) { // entry(..).or_default (the table itself is built after the walk)
            nclients++;
            ct.keys[f] = client;
            uint32_t *sr = cl + CLW * f;
            for (uint32_t k = 0; k < CLW; k++) sr[k] = 0;
            if (DIFF) {
              const uint32_t *svt = scr + L.sq;
              uint32_t rc = 0;
              for (uint32_t k = 0; k < nsv; k++)
                if (svt[2 * k] == client) rc = svt[2 * k + 1];
              sr[4] = rc;
            }
          }
          e = f;
          const uint32_t *sr = cl + CLW * e;
          nstored = sr[0];
          lkind = sr[1];
          lclock = sr[2];
          llen = sr[3];
          remote = sr[4];
          found = sr[5];
          count = sr[10];
          if (((uint64_t)nstored + nb) * 32ull > ALLOC_LIMIT || nsec >= cap.C) R.fail = F_BAIL;
          kb = 0xFFFFFFFFu;
          pure = 1;
          ssize = 0;
          j = 0;
          if (nb) st = R_BLOCK;
          else sec_end = true;
        }
      } else if (st == R_DRANGE) {
        // ---- one DeleteSet range (start, len)
        uint32_t rs, rl;
        bool c1, c2;
        q += R.var(q, rs, c1);
        q += R.var(q, rl, c2);
        if (!R.fail && (uint64_t)rs + rl > 0xFFFFFFFFull) R.fail = F_BAIL;
        if (!R.fail) {
          pos = q;
          dcanon &= c1 && c2;
          if (kr > 0 && rs < prev_e) dsq = false;
          prev_e = rs + rl;
          dsz += varlen(rs) + varlen(rl);
          if (++kr == nr) entry_end = true;
        }
      } else if (st == R_DENT) {
        // ---- DeleteSet entry header: client, range count
        q += R.var(q, dclient, cn);
        const uint32_t cp = q;
        q += R.var(q, nr, cn);
        if (!R.fail) {
          pos = q;
          cpos = cp;
          dcanon = cn;
          dsq = true;
          prev_e = 0;
          dsz = varlen(nr);
          kr = 0;
          if (nr) st = R_DRANGE;
          else entry_end = true;
        }
      } else if (st == R_NCL) {
        q += R.var(q, ncl, cn);
        if (!R.fail && ncl > cap.C) R.fail = F_BAIL;
        if (!R.fail) {
          pos = q;
          st = ncl ? R_SEC : R_NDS;
        }
      } else { // R_NDS
        q += R.var(q, nds, cn);
        if (!R.fail && DIFF && nds > cap.E) R.fail = F_BAIL;
        if (!R.fail) {
          pos = q;
          ids = 0;
          st = nds ? R_DENT : R_DONE;
        }
      }
      if (R.fail == F_SHORT) { // nothing consumed: the item is read again after the refill
        wait = true;
        continue;
      }
      if (R.fail) {
        bail = true;
        active = false;
        continue;
      }
      if (sec_end) {
        if (kb == 0xFFFFFFFFu) kb = pos;
        uint32_t *sr = sec + SECW * nsec++;
        sr[0] = e;
        sr[1] = kb;
        sr[2] = pos;
        sr[3] = pure;
        sr[4] = ssize;
        uint32_t *cr = cl + CLW * e;
        cr[0] = nstored;
        cr[1] = lkind | 0x100;
        cr[2] = lclock;
        cr[3] = llen;
        cr[5] = found;
        cr[10] = count;
        st = ++isec < ncl ? R_SEC : R_NDS;
      }
      if (entry_end) {
        if (DIFF) {
          if (!dsq) { // squash of a clone: general planner
            bail = true;
            active = false;
            continue;
          }
          uint32_t *r = de + DEW * ids;
          r[0] = dclient;
          r[1] = cpos;
          r[2] = pos;
          r[3] = nr;
          r[4] = 1u | (dcanon ? 2u : 0u);
          r[7] = varlen(dclient) + dsz;
        }
        st = ++ids < nds ? R_DENT : R_DONE;
      }
      if (st == R_DONE) active = false;
    }
    if (ps.stamps) t_stp += __builtin_amdgcn_s_memtime() - tq;
  }
  const uint64_t tf0 = ps.stamps ? __builtin_amdgcn_s_memtime() : 0;
  // ---- after the walk (out of the step loop: the calls below do not hold its registers):
  // hash tables replayed in yrs' insertion order, re-encoded slice sizes, the output plan
  if (d >= b.n_docs) return;
  if (!bail && st == R_DONE) {
    if (ncl && !ct.reserve(ncl, scr + L.ct_tmp)) bail = true;
    for (uint32_t f = 0; f < nclients && !bail; f++) {
      if (!ct.reserve(1, scr + L.ct_tmp)) bail = true;
      else ct.place(ct.keys[f], f);
    }
    if (DIFF) {
      for (uint32_t i = 0; i < nds && !bail; i++) {
        const uint32_t dc = de[DEW * i];
        if (!dt.reserve(1, scr + L.dt_tmp)) {
          bail = true;
          break;
        }
        const int f = dt.find(dc);
        if (f >= 0) { // replaced in place: the slot now names entry i
          for (uint32_t s = 0; s < dt.buckets; s++)
            if (dt.slot[s] == (uint32_t)f + 1) dt.slot[s] = i + 1;
          dt.keys[i] = dc;
        } else {
          dt.place(dc, i);
        }
      }
    }
    if (!bail) {
      uint64_t sz = 0;
      const uint32_t stt = plan_finish<DIFF>(scr, L, cap, ct, nsec, dt, false, 0u, sz);
      if (stt == PLAN_OVF) {
        bail = true;
      } else {
        if (b.frame && !stt) sz += 2 + varlen(sz); // y-sync message framing
        ps.big[d] = 0;
        ps.status[d] = (uint8_t)stt;
        ps.size[d] = stt ? 0 : sz;
      }
    }
  }
  if (bail) ps.big[d] = PLAN_REDO;
  if (ps.stamps) {
    uint64_t *o = ps.stamps + (size_t)d * 16;
    o[0] = t_ref;
    o[1] = t_stp;
    o[2] = __builtin_amdgcn_s_memtime() - tf0;
    o[3] = n_ref;
    o[4] = n_stp;
    o[5] = un;
    o[7] = 0xD1FF;
  }
}

// ------------------------------------------------------------------ wave planner
// k_plan_wave: the common-shape planner with ONE WAVEFRONT per document.  The ring planner
// above walks a document with one lane, so a wave runs 64 documents whose lanes sit on
// different item kinds: it is instruction-issue bound (~960 instructions per item step).
// Here all 64 lanes parse one document.  The v1 grammar interleaves raw string bytes with
// varints, so a ballot over continuation bits does not find block boundaries; a block's end is
// only known by parsing it.  A client section's blocks are parsed in windows of 64 chunks of
// 64 bytes (4 KB staged in LDS with 16-byte loads):
//   1 speculation: every lane parses blocks from the start of its own chunk (a guess; lane
//     0's start is the true boundary), recording the block starts it visits in a 64-bit mask
//     and the position where it leaves the chunk (its exit);
//   2 stitch: lane i's true entry is lane i-1's exit.  When that position is in lane i's mask
//     the two parses coincide from there on (a parse is a function of its start position), so
//     lane i's exit is right too; lanes whose entry is not in their mask parse again from it,
//     in rounds, until every lane agrees with its predecessor.  A parse from a wrong offset
//     falls back onto the true boundaries within a block or two, so one round is the norm;
//   3 the block starts at or after each lane's entry are its true blocks; a wave prefix sum of
//     their counts gives every block its index in the section, which ends after the block
//     count of its header (the parse past that point belongs to the next section header);
//   4 every lane walks its true blocks once more with the validation (canonical varints,
//     ASCII strings, info byte as re-encoded), summing clock lengths; a prefix sum gives each
//     block its clock; the lane holding the first block past the remote clock records it.
// The DeleteSet is varints only: a 512-byte window of it is split by a ballot over terminator
// bytes (bit 7 clear), a prefix sum gives every varint its index, one decode per varint start
// goes to LDS; the entry headers are then read in turn and each entry's ranges checked
// lane-parallel (squashed, canonical, no u32 overflow).
// It plans the ring planner's shapes (canonical blocks with Deleted / ASCII String content or
// GC, squashed DeleteSet entries, <= 8 clients and entries, u32 varints of <= 5 bytes) minus
// Skip blocks and zero-length items, and a block must fit one window; every other document is
// marked PLAN_REDO for k_plan.  It fills the same scratch records as plan_doc and ends in the
// same plan_finish, so its plans are byte-identical to the ring's and the general planner's.
constexpr uint32_t PW_WPB = 4;                   // documents (one wavefront each) per workgroup
constexpr uint32_t PW_C = 64;                    // chunk bytes per lane
constexpr uint32_t PW_BURN = 0;                  // bytes parsed before a chunk to fall onto the true blocks
constexpr uint32_t PW_SB = 64 * PW_C + 512 + 16; // block window bytes: 64 chunks + one block's slack + alignment
constexpr uint32_t PW_DB = 512;                  // DeleteSet window bytes (8 per lane)
constexpr uint32_t PW_SW = PW_SB / 4 + 4;        // block stage words (var_at reads 8 bytes at any p < PW_SB)
constexpr uint32_t PW_DW = PW_DB / 4 + 4;        // DeleteSet stage words, then values and metas
constexpr uint32_t PW_UW = PW_SW > PW_DW + 2 * PW_DB ? PW_SW : PW_DW + 2 * PW_DB;
constexpr uint32_t PW_FAIL = 0xFFFF0000u;        // exits >= this: the parse stopped
constexpr uint32_t PW_SHORT = 0xFFFFFFFEu;       // ...at the end of the staged bytes (more follow)
constexpr uint32_t PW_BAD = 0xFFFFFFFFu;         // ...on bytes that are not a planned block
constexpr uint32_t PW_NCL = 8, PW_NSV = 32, PW_NONE = 0xFFFFFFFFu;
static_assert(PW_NCL == 8, "small_caps(): 8 clients, 8 DeleteSet entries");

struct PwLds {
  uint32_t u[PW_UW];         // block stage | DeleteSet stage, values, metas (pos | canon << 16 | fine << 17 | n << 20)
  uint32_t svt[2 * PW_NSV];  // remote state vector entries (client, clock)
  uint32_t cl[CLW * PW_NCL]; // plan_doc's per-client records
  uint32_t sec[SECW * PW_NCL];
  uint32_t de[DEW * PW_NCL];
  uint32_t keys[PW_NCL];
};

struct PwB {
  uint32_t kind, len, info, ropos, rbytes;
  bool ok;
};
// One block at window byte p (Update::decode_block, yrs/src/update.rs:433-488, with
// ItemContent::decode of refs 1 / 4, block.rs:1786-1835): the position after it, or PW_SHORT /
// PW_BAD.  The block is a short program of fields read by one loop (the lanes of a wave parse
// different block kinds, so a branch per field kind would cost every lane every kind): 2 bits
// per field, low end first -- 0 varint, 1 varint + that many bytes, 2 parent info (1 = a named
// root: the two ID varints that follow become one string), 3 end.  FULL adds the plan checks
// (o.ok): canonical varints, the info byte as re-encoded (Item::info, block.rs:1363-1369: 0x10
// never, 0x20 only with a decoded parent_sub), parent info 0 / 1, ASCII strings (UTF-16 length
// == byte length), non-zero length.
template <bool FULL>
YM_INLINE uint32_t pw_block(const uint32_t *w, uint32_t p, uint32_t lim, bool more, PwB &o) {
  if (p >= lim) return more ? PW_SHORT : PW_BAD;
  const uint32_t info = lds_byte(w, p), ref = info & 15;
  // the content kinds planned here, tested first (a speculative parse rejects most wrong offsets
  // on their first byte): GC, Deleted (1), String (4); Skip (info 10) is the general planner's
  if (info != 0 && ref != 1 && ref != 4) return PW_BAD;
  const uint32_t no = info & 0x80 ? 2u : 0u, nr = info & 0x40 ? 2u : 0u;
  const bool par = info != 0 && (info & 0xC0) == 0, sub = par && (info & 0x20);
  const uint32_t content = ref == 4 ? 1u : 0u;
  uint32_t pat;
  if (info == 0) {
    pat = 0u | (3u << 2);
  } else {
    uint32_t sh = 2 * (no + nr); // origin / right origin: plain varints
    pat = 0;
    if (par) {
      pat |= 2u << sh; // parent info, then an ID's two varints (or the root name)
      sh += 6;
      if (sub) {
        pat |= 1u << sh;
        sh += 2;
      }
    }
    pat |= content << sh;
    pat |= 3u << (sh + 2);
  }
  uint32_t q = p + 1, fi = 0, v = 0, st = 0, ropos = q, roend = q;
  bool cn = true, pbad = false;
  for (;;) {
    const uint32_t k = pat & 3;
    if (k == 3) break;
    if (fi == no) ropos = q;
    if (fi == no + nr) roend = q;
    if (q >= lim) {
      st = more ? PW_SHORT : PW_BAD;
      break;
    }
    const VarR r = var_at(w, q, lim);
    if (!r.fine) {
      st = more && q + 5 > lim ? PW_SHORT : PW_BAD;
      break;
    }
    cn &= r.canon;
    v = r.v;
    q += r.n;
    if (k == 1) {
      if (v > lim - q) {
        st = more ? PW_SHORT : PW_BAD;
        break;
      }
      q += v;
    }
    pat >>= 2;
    if (k == 2) {
      pbad = v > 1;
      if (v == 1) pat = ((pat >> 4) << 2) | 1u; // the name string replaces the ID
    }
    fi++;
  }
  if (st) return st;
  o.info = info;
  o.kind = info == 0 ? BK_GC : BK_ITEM;
  o.len = v;
  o.ropos = ropos;
  o.rbytes = roend - ropos;
  if (FULL) {
    bool ok = cn && !pbad && v != 0 && !(info & 0x10) && !((info & 0x20) && (info & 0xC0));
    if (content && v > 1) { // String: ASCII (one byte: one UTF-16 unit whatever it is)
      uint32_t hi = 0;
      const uint32_t s0 = q - v, q0 = s0 >> 2, q1 = (q - 1) >> 2;
      for (uint32_t k = q0; k <= q1; k++) {
        uint32_t x = w[k];
        if (k == q0) x &= 0xFFFFFFFFu << (8 * (s0 & 3));
        if (k == q1 && (q & 3)) x &= 0xFFFFFFFFu >> (8 * (4 - (q & 3)));
        hi |= x;
      }
      ok = ok && !(hi & 0x80808080u);
    }
    o.ok = ok;
  }
  return q;
}
// Speculative parse of one lane's chunk [cs, ce) from p (cs <= p): the block starts it visits
// (mask) and where it leaves the chunk.  A parse that fails moves on by one byte, so the walk is
// a function N of the position (N(x) = the end of the block at x when x parses, else x + 1)
// and always leaves the chunk; from a true block start N follows the true blocks until one of
// them fails, which the validating walk finds.
// A lane's first parse starts PW_BURN bytes before its chunk (lane 0: at the true start), so a
// wrong offset has that long to fall onto the true blocks before the chunk begins.
YM_INLINE uint32_t pw_spec(const uint32_t *w, uint32_t p, uint32_t cs, uint32_t ce, uint32_t lim, bool more,
                           uint64_t &mask) {
  mask = 0;
  PwB o;
  while (p < ce) {
    if (p >= cs) mask |= 1ull << (p - cs);
    const uint32_t q = pw_block<false>(w, p, lim, more, o);
    p = q >= PW_FAIL ? p + 1 : q;
  }
  return p;
}

// The DeleteSet of one update (IdSet::decode, id_set.rs:412-426) from update byte P on, read
// by one wavefront: windows of PW_DB bytes staged in u (PW_DW + 2 PW_DB words); a ballot over
// terminator bytes (bit 7 clear) splits a window into varints, a prefix sum numbers them, one
// decode per varint start goes to LDS (value; position, canonical, fits-the-window flags,
// length); the entry headers are then read in turn and each entry's ranges checked lane-parallel
// (no u32 overflow; DIFF: squashed, canonical), its plan record written to de (DEW words, lane
// 0).  false: a shape for k_plan (malformed, unsquashed, more than capE entries).
template <bool DIFF>
__device__ __forceinline__ bool pw_deleteset(uint32_t *u, uint32_t *de, const uint8_t *up, uint32_t un, uint32_t P,
                                          uint32_t lane, uint32_t capE, uint32_t &nds) {
  const uintptr_t A0 = (uintptr_t)up;
  int32_t wb = 0;
  uint32_t lim = 0;
  bool more = false;
  auto stage = [&](uint32_t Q, uint32_t nbytes) {
    wsync(); // every lane is done with the previous stage
    const uintptr_t ab = (A0 + Q) & ~(uintptr_t)15;
    wb = (int32_t)(int64_t)(ab - A0);
    const uint32_t avail = (uint32_t)((int64_t)un - wb);
    lim = avail < nbytes ? avail : nbytes;
    more = avail > nbytes;
    const uint4 *src = (const uint4 *)ab;
    uint4 *dst = (uint4 *)u;
    const uint32_t n16 = (lim + 15) >> 4;
    for (uint32_t k = lane; k < n16; k += 64) dst[k] = src[k];
    wsync();
  };
  uint32_t *val = u + PW_DW, *meta = u + PW_DW + PW_DB;
  uint32_t nvar = 0, nfine = 0, kk = 0;
  bool fshort = false;
  auto ds_stage = [&](uint32_t Q) {
    stage(Q, PW_DB);
    const uint32_t off0 = (uint32_t)((int32_t)Q - wb), bq = 8 * lane;
    const uint64_t x = ((uint64_t)u[2 * lane + 1] << 32) | u[2 * lane];
    const uint32_t lo = off0 > bq ? (off0 - bq < 8 ? off0 - bq : 8u) : 0u;
    const uint32_t hi = lim > bq ? (lim - bq < 8 ? lim - bq : 8u) : 0u;
    const uint32_t vm = hi > lo ? ((1u << hi) - 1) & ~((1u << lo) - 1) : 0u;
    uint32_t tm = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) tm |= (uint32_t)((~x >> (8 * k + 7)) & 1) << k;
    tm &= vm;
    const uint32_t pt = shfl(tm, (int)((lane + 63) & 63));
    uint32_t sm = ((tm << 1) | (lane > 0 ? (pt >> 7) & 1 : 0u)) & 0xFF;
    if (off0 >= bq && off0 < bq + 8) sm |= 1u << (off0 - bq);
    sm &= vm;
    const uint32_t cnt = (uint32_t)__builtin_popcount(sm);
    const uint32_t inc = wincl(cnt, lane);
    uint32_t idx = inc - cnt, firstbad = PW_NONE, m = sm;
    while (m) {
      const uint32_t k = (uint32_t)__builtin_ctz(m);
      m &= m - 1;
      const VarR r = var_at(u, bq + k, lim);
      val[idx] = r.v;
      meta[idx] = (bq + k) | (r.canon ? 1u << 16 : 0u) | (r.fine ? 1u << 17 : 0u) | (r.n << 20);
      if (!r.fine && firstbad == PW_NONE) firstbad = idx;
      idx++;
    }
    nvar = rdlane(inc, 63);
    // the first varint that does not end inside the window: cut by the window end, or malformed
    uint32_t fb = firstbad;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = shfl(fb, (int)(lane ^ (uint32_t)o));
      fb = y < fb ? y : fb;
    }
    nfine = fb == PW_NONE ? nvar : fb;
    wsync();
    fshort = more && (nfine == nvar || (meta[nfine] & 0xFFFF) + 5 > lim);
    kk = 0;
  };
  // varints [kk, kk + n) readable in this window: restage at varint kk when the window cut
  // them; false = they are malformed or past the update's end (k_plan reports the error)
  auto ds_need = [&](uint32_t n) -> bool {
    if (kk + n <= nfine) return true;
    if (!fshort) return false;
    const uint32_t Q = kk < nvar ? (uint32_t)wb + (meta[kk] & 0xFFFF) : (uint32_t)wb + lim;
    ds_stage(Q);
    return kk + n <= nfine;
  };
  bool bail = false;
  nds = 0;
  ds_stage(P);
  if (!ds_need(1)) bail = true;
  else nds = val[kk++];
  if (DIFF && nds > capE) bail = true;
  for (uint32_t i = 0; i < nds && !bail; i++) {
    if (!ds_need(2)) {
      bail = true;
      break;
    }
    const uint32_t client = val[kk], nr = val[kk + 1];
    bool dcanon = (meta[kk + 1] >> 16) & 1;
    const uint32_t cpos = (uint32_t)wb + (meta[kk + 1] & 0xFFFF);
    uint32_t epos = cpos + (meta[kk + 1] >> 20);
    kk += 2;
    uint32_t dsz = varlen(nr), rr = nr, r0 = 0, prev_e = 0;
    while (rr) {
      if (kk + 2 > nfine && !ds_need(2)) {
        bail = true;
        break;
      }
      const uint32_t avail = (nfine - kk) / 2, m = rr < avail ? rr : avail;
      bool bad = false, unsq = false, cn = true;
      uint32_t sz = 0;
      for (uint32_t r = lane; r < m; r += 64) {
        const uint32_t s = val[kk + 2 * r], l = val[kk + 2 * r + 1];
        cn &= (meta[kk + 2 * r] >> 16) & (meta[kk + 2 * r + 1] >> 16) & 1;
        bad |= (uint64_t)s + l > 0xFFFFFFFFull;
        const uint32_t pe = r == 0 ? prev_e : val[kk + 2 * r - 2] + val[kk + 2 * r - 1];
        unsq |= (r0 + r > 0) && s < pe;
        sz += varlen(s) + varlen(l);
      }
      if (__ballot(bad) || (DIFF && __ballot(unsq))) { // overflow: k_plan; unsquashed: squash of a clone
        bail = true;
        break;
      }
      dcanon = dcanon && !__ballot(!cn);
      dsz += rdlane(wincl(sz, lane), 63);
      prev_e = val[kk + 2 * m - 2] + val[kk + 2 * m - 1];
      const uint32_t lm = meta[kk + 2 * m - 1];
      epos = (uint32_t)wb + (lm & 0xFFFF) + (lm >> 20);
      kk += 2 * m;
      rr -= m;
      r0 += m;
    }
    if (bail) break;
    if (DIFF && lane == 0) {
      uint32_t *r = de + DEW * i;
      r[0] = client;
      r[1] = cpos;
      r[2] = epos;
      r[3] = nr;
      r[4] = 1u | (dcanon ? 2u : 0u);
      r[5] = 0;
      r[6] = 0;
      r[7] = varlen(client) + dsz;
    }
  }
  wsync();
  return !bail;

}

// One document on one wavefront (all 64 lanes call it with the same d).
template <bool DIFF>
__device__ __forceinline__ void pw_plan_doc(const DiffBatch &b, const PlanScratch &ps, PwLds &S, uint32_t lane,
                                         uint32_t d) {
  if (b.ls_done && b.ls_done[d]) return; // the long-update grid path's (ylong.hip)
  if (b.pre_status && b.pre_status[d]) { // e.g. a y-sync message that is not SyncStep1
    if (lane == 0) {
      ps.big[d] = 0;
      ps.status[d] = b.pre_status[d];
      ps.size[d] = 0;
    }
    return;
  }
  const uint64_t o0 = b.upd_off[d], o1 = b.upd_off[d + 1];
  const uint8_t *up = b.bytes + o0;
  const uint32_t un = (uint32_t)(o1 - o0);
  uint32_t *scr = ps.small + (size_t)d * ps.small_words;
  const PlanCaps cap = small_caps();
  const PlanLayout L = plan_layout(cap);
  bool bail = o1 - o0 >= (1ull << 31);
  uint32_t nsv = 0;
  if (DIFF && !bail) { // remote state vector, decoded before the update (alt.rs:77-78), by lane 0
    uint32_t fl = 0;
    if (lane == 0) {
      const uint8_t *svp = b.sv + b.sv_off[d];
      const uint32_t svn = (uint32_t)((b.sv_end ? b.sv_end[d] : b.sv_off[d + 1]) - b.sv_off[d]);
      Cur s{svp, svn, 0};
      bool cn;
      uint32_t len = 0, clk, n = 0;
      uint64_t c;
      bool bl = rd_var_u32(s, len, cn) || (len && (uint64_t)buckets_for(len) * 17ull > ALLOC_LIMIT);
      for (uint32_t i = 0; i < len && !bl; i++) {
        if (rd_var_u64(s, c, cn) || rd_var_u32(s, clk, cn)) {
          bl = true;
          break;
        }
        if (c >> 32) continue; // no u32 block client can match it
        uint32_t k = 0;
        while (k < n && S.svt[2 * k] != (uint32_t)c) k++;
        if (k == n) {
          if (n == PW_NSV) {
            bl = true;
            break;
          }
          n++;
        }
        S.svt[2 * k] = (uint32_t)c; // a client listed twice keeps its last clock (HashMap::insert)
        S.svt[2 * k + 1] = clk;
      }
      fl = (bl ? 1u : 0u) | (n << 8);
    }
    fl = rdlane(pin(fl), 0);
    bail = fl & 1;
    nsv = fl >> 8;
    wsync();
  }

  // ---- staging: window byte p <-> update byte wb + p (wb: the 16-byte aligned base)
  const uintptr_t A0 = (uintptr_t)up;
  int32_t wb = 0;
  uint32_t lim = 0;
  bool more = false;
  auto stage = [&](uint32_t P, uint32_t nbytes) {
    wsync(); // every lane is done with the previous stage
    const uintptr_t ab = (A0 + P) & ~(uintptr_t)15;
    wb = (int32_t)(int64_t)(ab - A0);
    const uint32_t avail = (uint32_t)((int64_t)un - wb);
    lim = avail < nbytes ? avail : nbytes;
    more = avail > nbytes;
    const uint4 *src = (const uint4 *)ab;
    uint4 *dst = (uint4 *)S.u;
    const uint32_t n16 = (lim + 15) >> 4;
    for (uint32_t k = lane; k < n16; k += 64) dst[k] = src[k];
    wsync();
  };
  // a header varint (re-emitted from its value: canonical form not required) at update byte P
  auto hdr_var = [&](uint32_t &P, uint32_t &v) -> bool {
    uint32_t p = (uint32_t)((int32_t)P - wb);
    if (p + 16 > lim && more) {
      stage(P, PW_SB);
      p = (uint32_t)((int32_t)P - wb);
    }
    const VarR r = var_at(S.u, p, lim);
    if (p >= lim || !r.fine) return false;
    v = r.v;
    P += r.n;
    return true;
  };

  uint32_t P = 0, ncl = 0, nclients = 0, nsec = 0, nds = 0;
  uint32_t n_win = 0, n_round = 0; // diagnostic stamps (YMERGE_STAMPS): windows, stitch rounds
  if (!bail) {
    stage(0, PW_SB);
    if (!hdr_var(P, ncl) || ncl > cap.C) bail = true;
  }
  // ---- client sections
  for (uint32_t isec = 0; isec < ncl && !bail; isec++) {
    uint32_t nb, client, clock;
    if (!hdr_var(P, nb) || !hdr_var(P, client) || !hdr_var(P, clock)) {
      bail = true;
      break;
    }
    uint32_t e = nclients;
    for (uint32_t f = 0; f < nclients; f++)
      if (S.keys[f] == client) {
        e = f;
        break;
      }
    if (e == nclients) { // entry(..).or_default (the hash table is replayed after the walk)
      if (nclients == PW_NCL) {
        bail = true;
        break;
      }
      nclients++;
      wsync();
      if (lane < CLW) {
        uint32_t v = 0;
        if (DIFF && lane == 4)
          for (uint32_t k = 0; k < nsv; k++)
            if (S.svt[2 * k] == client) v = S.svt[2 * k + 1];
        S.cl[CLW * e + lane] = v;
      }
      if (lane == 0) S.keys[e] = client;
      wsync();
    }
    uint32_t *cr = S.cl + CLW * e;
    const uint32_t nstored = cr[0], remote = cr[4];
    uint32_t lkind = cr[1] & 0xFF, lclock = cr[2], llen = cr[3], found = cr[5], count = cr[10];
    if (((uint64_t)nstored + nb) * 32ull > ALLOC_LIMIT || nsec >= cap.C) {
      bail = true;
      break;
    }
    uint32_t kb = PW_NONE, R = nb;
    uint64_t clk = clock;
    while (R && !bail) {
      // ---- one window of this section's blocks, from the true block start P
      stage(P, PW_SB);
      n_win++;
      const uint32_t off0 = (uint32_t)((int32_t)P - wb);
      const uint32_t cs = off0 + PW_C * lane, ce = cs + PW_C;
      uint64_t mask;
      uint32_t ex = pw_spec(S.u, lane == 0 ? cs : (cs - PW_BURN > off0 ? cs - PW_BURN : off0), cs, ce, lim, more,
                            mask);
      uint32_t t = cs;
      for (;;) { // stitch: until every lane agrees with its predecessor's exit
        const uint32_t pex = shfl(ex, (int)((lane + 63) & 63));
        t = lane == 0 ? off0 : pex;
        const bool cons = lane == 0 || t >= ce || ((mask >> (t - cs)) & 1);
        if (!__ballot(!cons)) break;
        n_round++;
        if (!cons) { // parse again from the entry until it meets the chain already parsed
          uint64_t nm = 0;
          uint32_t p = t;
          PwB o;
          while (p < ce) {
            if ((mask >> (p - cs)) & 1) { // merged: the rest of the chain and the exit stand
              nm |= mask & (~0ull << (p - cs));
              p = ex;
              break;
            }
            nm |= 1ull << (p - cs);
            const uint32_t q = pw_block<false>(S.u, p, lim, more, o);
            p = q >= PW_FAIL ? p + 1 : q;
          }
          mask = nm;
          ex = p;
        }
      }
      // this lane's block starts from its true entry on (true blocks up to the first that fails)
      mask = t >= ce ? 0ull : mask & (~0ull << (t - cs));
      const uint32_t cnt = (uint32_t)__builtin_popcountll(mask);
      const uint32_t inc = wincl(cnt, lane), exc = inc - cnt, tot = rdlane(inc, 63);
      const uint32_t nw0 = R < tot ? R : tot;
      // ---- validating walk of the true blocks, clock lengths
      const uint32_t k = exc < nw0 ? (cnt < nw0 - exc ? cnt : nw0 - exc) : 0u;
      uint32_t p = t, lkd = 0, lcl = 0, lln = 0, j = 0, fst = 0;
      uint64_t sum = 0;
      for (; j < k; j++) {
        PwB o;
        const uint32_t q = pw_block<true>(S.u, p, lim, more, o);
        if (q >= PW_FAIL || !o.ok) {
          fst = q == PW_SHORT ? PW_SHORT : PW_BAD;
          break;
        }
        lkd = o.kind;
        lcl = (uint32_t)sum;
        lln = o.len;
        sum += o.len;
        p = q;
      }
      // the first block of the window that fails: past the stage -> the window ends before it;
      // not a planned block -> k_plan
      uint32_t nw = nw0;
      const uint64_t fm = __ballot(fst != 0);
      if (fm) {
        const uint32_t fl = (uint32_t)__builtin_ctzll(fm);
        const uint32_t gf = rdlane(exc + j, fl);
        if (rdlane(fst, fl) == PW_BAD || gf == 0) {
          bail = true;
          break;
        }
        nw = gf;
      }
      if (exc >= nw) { // blocks past the window's last committed one
        sum = 0;
        j = 0;
      }
      if (__ballot(sum >= (1ull << 25))) { // keeps the wave's clock sums in u32 (longer runs: k_plan)
        bail = true;
        break;
      }
      const uint32_t kw = j; // blocks this lane commits
      const uint32_t s32 = (uint32_t)sum;
      const uint32_t cinc = wincl(s32, lane), cexc = cinc - s32, ctot = rdlane(cinc, 63);
      if (clk + ctot > 0xFFFFFFFFull) { // clock += len would overflow (a debug-build panic)
        bail = true;
        break;
      }
      const uint32_t lastl = (uint32_t)__builtin_ctzll(__ballot(kw > 0 && exc + kw == nw));
      lkind = rdlane(lkd, lastl);
      lclock = (uint32_t)clk + rdlane(cexc + lcl, lastl);
      llen = rdlane(lln, lastl);
      const uint32_t pend = rdlane(p, lastl);
      if (DIFF) {
        if (found) {
          if (kb == PW_NONE) kb = P; // a section after the one holding the client's first diff block
          count += nw;
        } else {
          // Update::encode_diff: the first block whose end passes the remote clock
          const uint64_t fmask = __ballot(kw > 0 && clk + cexc + sum > (uint64_t)remote);
          if (fmask) {
            const uint32_t fl = (uint32_t)__builtin_ctzll(fmask);
            uint32_t jf = 0, kbw = 0;
            if (lane == fl) {
              uint32_t q = t, c = (uint32_t)clk + cexc;
              for (uint32_t jj = 0; jj < kw; jj++) {
                PwB o;
                const uint32_t qn = pw_block<true>(S.u, q, lim, more, o);
                if ((uint64_t)c + o.len > remote) {
                  const uint32_t off = remote > c ? remote - c : 0u;
                  const uint32_t blen = qn - q;
                  uint32_t sz;
                  if (off == 0) {
                    sz = blen;
                  } else if (o.kind != BK_ITEM) {
                    sz = 1 + varlen(o.len - off);
                  } else { // ItemSlice::encode with an offset (see the ring planner)
                    const uint32_t rest = o.len - off;
                    sz = 1 + varlen(client) + varlen(c + off - 1) + o.rbytes + varlen(rest) +
                         ((o.info & 15) == 4 ? rest : 0u);
                  }
                  uint32_t *sr = S.cl + CLW * e;
                  sr[6] = (uint32_t)wb + q;
                  sr[7] = c;
                  sr[8] = o.len;
                  sr[9] = off;
                  sr[11] = sz;
                  if (off == 0) {
                    sr[14] = 1;
                  } else if (o.kind == BK_ITEM) {
                    const uint32_t has_ps = (o.info & 0xE0) == 0x20 ? 1u : 0u;
                    sr[12] = (uint32_t)wb + o.ropos;
                    sr[13] = o.rbytes | ((o.info & 15) << 8) | (has_ps << 12) | ((qn - o.ropos) << 16);
                    sr[14] = 2;
                  }
                  jf = jj;
                  kbw = qn;
                  break;
                }
                c += o.len;
                q = qn;
              }
            }
            jf = rdlane(pin(jf), fl);
            kbw = rdlane(pin(kbw), fl);
            wsync();
            found = 1;
            count = nw - (rdlane(exc, fl) + jf); // the found block and every later one of the window
            kb = (uint32_t)wb + kbw;
          }
        }
      }
      R -= nw;
      clk += ctot;
      P = (uint32_t)wb + pend;
    }
    if (bail) break;
    // ---- section record (plan_doc's sec / cl updates)
    if (kb == PW_NONE) kb = P;
    wsync();
    if (lane == 0) {
      uint32_t *sr = S.sec + SECW * nsec;
      sr[0] = e;
      sr[1] = kb;
      sr[2] = P;
      sr[3] = 1;
      sr[4] = P - kb;
      cr[0] = nstored + nb;
      cr[1] = lkind | 0x100;
      cr[2] = lclock;
      cr[3] = llen;
      cr[5] = found;
      cr[10] = count;
    }
    nsec++;
    wsync();
  }

  // ---- DeleteSet
  if (!bail) bail = !pw_deleteset<DIFF>(S.u, S.de, up, un, P, lane, cap.E, nds);

  // ---- the plan (lane 0): scratch records, hash tables replayed in yrs' insertion order
  if (lane != 0) return;
  if (!bail) {
    for (uint32_t f = 0; f < nclients; f++) {
      scr[L.ct_keys + f] = S.keys[f];
      for (uint32_t k = 0; k < CLW; k++) scr[L.cl + CLW * f + k] = S.cl[CLW * f + k];
    }
    for (uint32_t s = 0; s < nsec * SECW; s++) scr[L.sec + s] = S.sec[s];
    if (DIFF)
      for (uint32_t s = 0; s < nds * DEW; s++) scr[L.de + s] = S.de[s];
    GHB ct{scr + L.ct_slot, scr + L.ct_keys, L.BC, 0, 0, 0};
    GHB dt{scr + L.dt_slot, scr + L.dt_keys, L.BE, 0, 0, 0};
    if (ncl && !ct.reserve(ncl, scr + L.ct_tmp)) bail = true;
    for (uint32_t f = 0; f < nclients && !bail; f++) {
      if (!ct.reserve(1, scr + L.ct_tmp)) bail = true;
      else ct.place(ct.keys[f], f);
    }
    if (DIFF) {
      const uint32_t *de = scr + L.de;
      for (uint32_t i = 0; i < nds && !bail; i++) {
        const uint32_t dc = de[DEW * i];
        if (!dt.reserve(1, scr + L.dt_tmp)) {
          bail = true;
          break;
        }
        const int f = dt.find(dc);
        if (f >= 0) { // replaced in place: the slot now names entry i
          for (uint32_t s = 0; s < dt.buckets; s++)
            if (dt.slot[s] == (uint32_t)f + 1) dt.slot[s] = i + 1;
          dt.keys[i] = dc;
        } else {
          dt.place(dc, i);
        }
      }
    }
    if (!bail) {
      uint64_t sz = 0;
      const uint32_t stt = plan_finish<DIFF>(scr, L, cap, ct, nsec, dt, false, 0u, sz);
      if (stt == PLAN_OVF) {
        bail = true;
      } else {
        if (b.frame && !stt) sz += 2 + varlen(sz); // y-sync message framing
        ps.big[d] = 0;
        ps.status[d] = (uint8_t)stt;
        ps.size[d] = stt ? 0 : sz;
      }
    }
  }
  if (bail) ps.big[d] = PLAN_REDO;
  if (ps.stamps) {
    uint64_t *o = ps.stamps + (size_t)d * 16;
    o[0] = n_win;
    o[1] = n_round;
    o[2] = bail ? 1 : 0;
    o[5] = un;
    o[7] = 0xD1FE;
  }
}


// Documents of >= PW_MIN bytes (listed by k_plan_lane; every document when ps.wave_list is
// null), a wavefront each, grid-stride.
template <bool DIFF>
__global__ void __launch_bounds__(64 * PW_WPB) k_plan_wave(DiffBatch b, PlanScratch ps) {
  ym_set_grammar(b.v1x);
  __shared__ __align__(16) PwLds lds_all[PW_WPB];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t n = ps.wave_list ? *ps.wave_n : b.n_docs;
  for (uint32_t i = blockIdx.x * PW_WPB + wv; i < n; i += gridDim.x * PW_WPB)
    pw_plan_doc<DIFF>(b, ps, lds_all[wv], lane, ps.wave_list ? ps.wave_list[i] : i);
}

// k_plan_lane: the ring planner's lane-per-document walk (a lane per document is the
// cheapest walk in parse steps: a wavefront per document needs ~10x more, k_plan_wave above)
// without the two costs that held the ring planner at ~570 VALU + ~450 SALU instructions per
// item step (SQ counters, profiles/r04/r04h_*): per-field branches that the 64 documents of a
// wave take differently (every step paid for every kind), and the DeleteSet walked range by
// range in the same loop.
//   * A block of the common kinds (GC; an Item with an origin and / or right origin and
//     Deleted or String content) is parsed straight-line from a 32-byte window of its ring:
//     per-byte masks (varint terminators, zero bytes, bytes >= 16) with a multiply per dword,
//     the content length's end as the n-th terminator, the canonical-varint checks as mask
//     algebra, the ASCII check as one mask test.  Everything else -- section headers,
//     parent-form or re-encoded blocks, blocks longer than the window, a section's last block,
//     the client's first diff block, an entry's last range -- takes the full step (one
//     field-program loop).
//   * A DeleteSet range (two varints) likewise, from a 16-byte window.
//   * The full step is batched: a lane that needs it waits until LP_SLOW lanes of its wave do
//     (or none can take a fast step), so the wave runs it once for many lanes.
// Same shapes, records and plans as the ring planner.
template <bool DIFF>
__global__ void __launch_bounds__(RING_NT) k_plan_lane(DiffBatch b, PlanScratch ps) {
  ym_set_grammar(b.v1x);
  __shared__ __align__(16) uint32_t ring_lds[RING_NT * RING_STRIDE / 4];
  const uint32_t t = threadIdx.x;
  const uint32_t d = blockIdx.x * RING_NT + t;
  uint32_t *row = ring_lds + t * (RING_STRIDE / 4);
  bool active = d < b.n_docs;
  if (active && b.pre_status && b.pre_status[d]) { // e.g. a y-sync message that is not SyncStep1
    ps.big[d] = 0;
    ps.status[d] = b.pre_status[d];
    ps.size[d] = 0;
    active = false;
  }
  if (active && b.ls_done && b.ls_done[d]) active = false; // the long-update grid path's (ylong.hip)
  if (active && ps.wave_list && b.upd_off[d + 1] - b.upd_off[d] >= PW_MIN) { // one long update: k_plan_wave
    ps.big[d] = PLAN_WAVE;
    ps.wave_list[atomicAdd(ps.wave_n, 1u)] = d;
    active = false;
  }
  const uint8_t *up = nullptr, *svp = nullptr;
  uint32_t un = 0, svn = 0, nsv = 0;
  uint32_t *scr = nullptr;
  const PlanCaps cap = small_caps();
  const PlanLayout L = plan_layout(cap);
  bool bail = false;
  if (active) {
    const uint64_t o0 = b.upd_off[d], o1 = b.upd_off[d + 1];
    up = b.bytes + o0;
    un = (uint32_t)(o1 - o0);
    if (o1 - o0 >= (1ull << 31)) bail = true;
    scr = ps.small + (size_t)d * ps.small_words;
    if (DIFF && !bail) { // remote state vector, decoded before the update (alt.rs:77-78)
      svp = b.sv + b.sv_off[d];
      svn = (uint32_t)((b.sv_end ? b.sv_end[d] : b.sv_off[d + 1]) - b.sv_off[d]);
      // entries with a u32 client id go to a small table (the sq region: unsquashed ranges
      // are the general planner's); a client listed twice keeps its last clock (HashMap::insert)
      Cur s{svp, svn, 0};
      bool cn;
      uint32_t len = 0, clk;
      uint64_t c;
      if (rd_var_u32(s, len, cn) || (len && (uint64_t)buckets_for(len) * 17ull > ALLOC_LIMIT)) bail = true;
      uint32_t *svt = scr + L.sq;
      for (uint32_t i = 0; i < len && !bail; i++) {
        if (rd_var_u64(s, c, cn) || rd_var_u32(s, clk, cn)) {
          bail = true;
          break;
        }
        if (c >> 32) continue;
        uint32_t k = 0;
        while (k < nsv && svt[2 * k] != (uint32_t)c) k++;
        if (k == nsv) {
          if (nsv == cap.R / 2) {
            bail = true;
            break;
          }
          nsv++;
        }
        svt[2 * k] = (uint32_t)c;
        svt[2 * k + 1] = clk;
      }
    }
    if (bail) active = false;
  }
  GHB ct{scr + L.ct_slot, scr + L.ct_keys, L.BC, 0, 0, 0};
  GHB dt{scr + L.dt_slot, scr + L.dt_keys, L.BE, 0, 0, 0};
  uint32_t *cl = scr + L.cl, *sec = scr + L.sec, *de = scr + L.de;
  uint32_t st = R_NCL, pos = 0, ncl = 0, isec = 0, nb = 0, j = 0, client = 0, clock = 0, nclients = 0;
  // current section (plan_doc's per-client record, kept in registers while the section runs)
  uint32_t e = 0, nstored = 0, lkind = 0, lclock = 0, llen = 0, remote = 0, found = 0, count = 0, kb = 0, pure = 1,
           ssize = 0, nsec = 0;
  // DeleteSet
  uint32_t nds = 0, ids = 0, dclient = 0, cpos = 0, nr = 0, kr = 0, prev_e = 0, dsz = 0;
  bool dcanon = true, dsq = true;
  RingRd R{row, (uint64_t)up, 0, 0, (uint64_t)up + un, un, F_OK, 0, 0};
  bool have = false, wait = false, need_slow = false;
  const uint32_t lp_slow = (ps.lane_dbg >> 8) & 0xFF ? (ps.lane_dbg >> 8) & 0xFF : LP_SLOW; // (diagnostic overrides)
  const uint32_t ring_steps = (ps.lane_dbg >> 16) & 0xFF ? (ps.lane_dbg >> 16) & 0xFF : LP_STEPS;

  // diagnostic stamps (wave time): refill, steps, finish; refill rounds, step iterations
  uint64_t t_ref = 0, t_stp = 0, n_ref = 0, n_stp = 0, tq = ps.stamps ? __builtin_amdgcn_s_memtime() : 0;
  for (;;) {
    if (!__any(active)) break;
    if (ps.stamps) tq = __builtin_amdgcn_s_memtime();
    // ---- refill point: lanes that ran short, or are within 64 bytes of their ring's end
    const uint64_t a0 = R.sbase + pos;
    if (active && (!have || wait || (a0 + 64 > R.rb + RING && R.rb + RING < R.send))) {
      if (have && wait && R.rb == (a0 & ~15ull)) { // an item longer than a fresh ring
        bail = true;
        active = false;
      } else {
        R.rb = a0 & ~15ull;
        const uint4 *q = (const uint4 *)R.rb;
        uint4 *dst = (uint4 *)row;
#pragma unroll
        for (uint32_t g = 0; g < RING / 16; g += RING_G) { // groups of 16-byte loads
          uint4 x[RING_G];
#pragma unroll
          for (uint32_t k = 0; k < RING_G; k++)
            x[k] = R.rb + 16 * (g + k) < R.send ? q[g + k] : make_uint4(0, 0, 0, 0);
#pragma unroll
          for (uint32_t k = 0; k < RING_G; k++) dst[g + k] = x[k];
        }
        R.rend = R.rb + RING < R.send ? R.rb + RING : R.send;
        R.sync_rel();
        have = true;
        wait = false;
      }
    }
    if (ps.stamps) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      t_ref += now - tq;
      tq = now;
      n_ref++;
    }
    for (uint32_t step = 0; step < ring_steps; step++) {
      const bool can = active && !wait;
      if (!__any(can)) break;
      if (ps.stamps) n_stp++;
      bool fast_done = false;
      if (can && !need_slow && st == R_BLOCK && !(ps.lane_dbg & 1)) {
        // ---- fast step: a block of the common kinds, straight-line from a 32-byte window of the
        //      ring (every lane runs the same instructions whatever its block's kind)
        const int32_t o = (int32_t)pos - R.rbq;
        if (!(o >= 0 && o + 36 <= (int32_t)RING_STRIDE && ((int32_t)pos + 32 <= R.rendq || R.rendq == (int32_t)un))) {
          wait = true; // the window runs past the ring: refill first
        } else {
          const uint32_t *wr = row + (o >> 2);
          const uint32_t sh = (uint32_t)o & 3;
          uint32_t x[8];
          {
            uint32_t a[9];
#pragma unroll
            for (int k = 0; k < 9; k++) a[k] = wr[k];
#pragma unroll
            for (int k = 0; k < 8; k++) x[k] = __builtin_amdgcn_alignbyte(a[k + 1], a[k], sh);
          }
          // byte masks, bit i = window byte i: varint terminators (bit 7 clear), zero bytes,
          // bytes of 16 and more (their low 7 bits); one multiply gathers a dword's four bits
          uint32_t T0 = 0, Z = 0, G = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const uint32_t dw = x[k];
            const uint32_t nz = (((dw & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | dw) & 0x80808080u;
            const uint32_t ge = ((dw & 0x70707070u) + 0x70707070u) & 0x80808080u;
            T0 |= (((((~dw & 0x80808080u) >> 7) * 0x204081u) >> 21) & 0xFu) << (4 * k);
            Z |= (((((~nz & 0x80808080u) >> 7) * 0x204081u) >> 21) & 0xFu) << (4 * k);
            G |= ((((ge >> 7) * 0x204081u) >> 21) & 0xFu) << (4 * k);
          }
          const uint32_t info = x[0] & 0xFF, ref = info & 15;
          const bool gc = info == 0, str = !gc && ref == 4;
          // GC, or an Item with an origin and / or a right origin (no parent info), Deleted or
          // String content, info byte as re-encoded (no 0x10; 0x20 only with a parent)
          const bool shape = gc || ((info & 0x30) == 0 && (info & 0xC0) != 0 && (ref == 1 || ref == 4));
          const uint32_t nv = gc ? 1u : (info & 0x80 ? 2u : 0u) + (info & 0x40 ? 2u : 0u) + 1u;
          const uint32_t T = T0 & ~1u, B = T0 | 1u; // B: where a varint may start after
          uint32_t tt = T, s = 0;
#pragma unroll
          for (uint32_t k = 1; k < 5; k++) { // s = end of the varint before the last (0: info)
            const uint32_t c = (uint32_t)__builtin_ctz(tt | 0x80000000u);
            s = k < nv ? c : s;
            tt = k < nv ? tt & (tt - 1) : tt;
          }
          const uint32_t e = tt ? (uint32_t)__builtin_ctz(tt) : 32u; // end of the content length
          const uint32_t R1 = e < 31 ? (2u << e) - 2u : 0xFFFFFFFEu;
          // canonical varints only (the block is copied verbatim): a multi-byte varint does not
          // end in a zero byte, none is longer than 5 bytes, a 5-byte one ends below 16
          const uint32_t multi = T & R1 & ~(B << 1);
          const uint32_t ge5 = multi & ~(B << 2) & ~(B << 3) & ~(B << 4);
          const bool canon = ((multi & Z) | (ge5 & ~(B << 5)) | (ge5 & G)) == 0;
          const uint32_t n = e - s;
          const uint64_t xv = ring_read8(row, (uint32_t)o + (s < 31 ? s + 1 : 0u));
          const uint64_t xm = xv & (n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1));
          const uint32_t len = (uint32_t)((xm & 0x7F) | ((xm >> 1) & 0x3F80) | ((xm >> 2) & 0x1FC000) |
                                          ((xm >> 3) & 0xFE00000) | ((xm >> 4) & 0x7F0000000ull));
          const bool fits = !str || (e < 32 && len <= 31 - e);
          const uint32_t pm = str && fits && len > 1 ? ((1u << len) - 1u) << (e + 1) : 0u;
          const uint32_t blen = e + 1 + (str ? len : 0u);
          bool fast = shape && e < 32 && canon && len != 0 && fits && (pm & ~T0) == 0 && blen <= un - pos &&
                      (uint64_t)clock + len <= 0xFFFFFFFFull && j + 1 < nb;
          if (DIFF) fast = fast && (found || clock + len <= remote); // the first diff block: the full step
          if (fast) {
            nstored++;
            lkind = gc ? BK_GC : BK_ITEM;
            lclock = clock;
            llen = len;
            if (DIFF && found) {
              if (kb == 0xFFFFFFFFu) kb = pos;
              count++;
              ssize += blen;
            }
            clock += len;
            pos += blen;
            j++;
            fast_done = true;
          } else {
            need_slow = true;
          }
        }
      } else if (can && !need_slow && st == R_DRANGE && kr + 1 < nr && !(ps.lane_dbg & 1)) {
        // ---- fast step: one DeleteSet range (start, length), two varints of a 16-byte window
        const int32_t o = (int32_t)pos - R.rbq;
        if (!(o >= 0 && o + 20 <= (int32_t)RING_STRIDE && ((int32_t)pos + 16 <= R.rendq || R.rendq == (int32_t)un))) {
          wait = true;
        } else {
          const uint32_t *wr = row + (o >> 2);
          const uint32_t sh = (uint32_t)o & 3;
          const uint32_t a0 = wr[0], a1 = wr[1], a2 = wr[2], a3 = wr[3], a4 = wr[4];
          const uint32_t x0 = __builtin_amdgcn_alignbyte(a1, a0, sh), x1 = __builtin_amdgcn_alignbyte(a2, a1, sh);
          const uint32_t x2 = __builtin_amdgcn_alignbyte(a3, a2, sh), x3 = __builtin_amdgcn_alignbyte(a4, a3, sh);
          const uint64_t lo = (uint64_t)x0 | ((uint64_t)x1 << 32), hi = (uint64_t)x2 | ((uint64_t)x3 << 32);
          const uint64_t tl = ~lo & 0x8080808080808080ull, th = ~hi & 0x8080808080808080ull;
          const uint32_t e1 = (uint32_t)__builtin_ctzll(tl | (1ull << 63)) >> 3; // 7: none in the low 8 bytes
          const uint32_t s2 = e1 + 1;                                             // second varint's start (<= 8)
          const uint64_t y = s2 >= 8 ? hi : (lo >> (8 * s2)) | (s2 ? hi << (64 - 8 * s2) : 0ull);
          const uint64_t ty = ~y & 0x8080808080808080ull;
          const uint32_t n2 = ((uint32_t)__builtin_ctzll(ty | (1ull << 63)) >> 3) + 1;
          const uint32_t n1 = e1 + 1;
          auto dec = [](uint64_t x, uint32_t n) -> uint32_t {
            const uint64_t xm = x & (n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1));
            return (uint32_t)((xm & 0x7F) | ((xm >> 1) & 0x3F80) | ((xm >> 2) & 0x1FC000) | ((xm >> 3) & 0xFE00000) |
                              ((xm >> 4) & 0x7F0000000ull));
          };
          const uint32_t rs = dec(lo, n1), rl = dec(y, n2);
          const uint32_t l1 = (uint32_t)(lo >> (8 * (n1 - 1))) & 0xFF, l2 = (uint32_t)(y >> (8 * (n2 - 1))) & 0xFF;
          const bool c1 = n1 == 1 || (l1 != 0 && (n1 < 5 || l1 < 16)), c2 = n2 == 1 || (l2 != 0 && (n2 < 5 || l2 < 16));
          const bool fine = n1 <= 5 && n2 <= 5 && n1 + n2 <= un - pos;
          const bool fast = fine && (uint64_t)rs + rl <= 0xFFFFFFFFull && (kr == 0 || rs >= prev_e || !DIFF);
          if (fast) {
            pos += n1 + n2;
            dcanon &= c1 && c2;
            if (kr > 0 && rs < prev_e) dsq = false;
            prev_e = rs + rl;
            dsz += varlen(rs) + varlen(rl);
            kr++;
            fast_done = true;
          } else {
            need_slow = true;
          }
        }
      } else if (can && st != R_BLOCK && !need_slow) {
        need_slow = true;
      } else if (can && (ps.lane_dbg & 1)) {
        need_slow = true;
      }
      // ---- full step (section headers, other block shapes, a section's last block, the
      //      client's first diff block), batched: it runs once enough lanes wait for it or no
      //      lane made progress, so a wave pays for it once per LP_SLOW lanes, not once per step
      const uint64_t slow_m = __ballot(can && need_slow);
      if (!slow_m) continue;
      if ((uint32_t)__builtin_popcountll(slow_m) < lp_slow && __ballot(fast_done)) continue;
      if (!(can && need_slow)) continue;
      need_slow = false;
      R.fail = F_OK;
      bool cn, sec_end = false, entry_end = false;
      // ---- the item's field program: one loop reads the varints of every item kind (lanes of
      //      a wave sit on different kinds -- string blocks, DeleteSet ranges, headers -- and run
      //      the same instructions); 2 bits per field, low end first: 0 varint, 1 varint + that
      //      many bytes, 2 parent info (1: the ID's two varints become the root name), 3 end
      uint32_t q = pos, info = 0, pat, no = 0, nr2 = 0;
      if (st == R_BLOCK) {
        info = (uint32_t)(R.at(q) & 0xFF);
        q++;
        const uint32_t ref = info & 15;
        if (info == 0 || info == 10) {
          pat = 0u | (3u << 2); // GC / Skip: length
        } else {
          if (ref != 1 && ref != 4 && !R.fail) R.fail = F_BAIL; // cold content kinds: general planner
          no = info & 0x80 ? 2u : 0u;
          nr2 = info & 0x40 ? 2u : 0u;
          uint32_t sh = 2 * (no + nr2);
          pat = 0;
          if ((info & 0xC0) == 0) {
            pat |= 2u << sh;
            sh += 6;
            if (info & 0x20) {
              pat |= 1u << sh;
              sh += 2;
            }
          }
          pat |= (ref == 4 ? 1u : 0u) << sh;
          pat |= 3u << (sh + 2);
        }
      } else {
        pat = st == R_SEC ? 3u << 6 : (st == R_DENT || st == R_DRANGE) ? 3u << 4 : 3u << 2;
      }
      uint32_t fi = 0, v = 0, f0 = 0, f1 = 0, f2 = 0, ropos = q, roend = q, p1 = q, ncan = 0;
      bool pbad = false;
      for (;;) {
        const uint32_t k = pat & 3;
        if (k == 3 || R.fail) break;
        if (fi == no) ropos = q;
        if (fi == no + nr2) roend = q;
        if (fi == 1) p1 = q;
        const uint32_t n = R.var(q, v, cn);
        if (R.fail) break;
        ncan |= (cn ? 0u : 1u) << fi;
        q += n;
        f0 = fi == 0 ? v : f0;
        f1 = fi == 1 ? v : f1;
        f2 = fi == 2 ? v : f2;
        if (k == 1) {
          if (v > un - q) {
            R.fail = F_BAIL;
            break;
          }
          q += v;
        }
        pat >>= 2;
        if (k == 2) {
          pbad = v > 1;
          if (v == 1) pat = ((pat >> 4) << 2) | 1u; // the name string replaces the ID
        }
        fi++;
      }
      if (st == R_BLOCK) {
        // ---- one block (Update::decode_block, update.rs:433-488 + ItemContent::decode)
        const uint32_t kind = info == 0 ? BK_GC : info == 10 ? BK_SKIP : BK_ITEM, len = v;
        const uint32_t rbytes = roend - ropos;
        bool reenc = ncan != 0;
        if (kind == BK_ITEM) {
          // 0x10 never re-emitted; 0x20 only when parent_sub was decoded; parent info 0 / 1
          reenc |= pbad || (info & 0x10) || ((info & 0x20) && (info & 0xC0));
          if ((info & 15) == 4 && !R.fail && len > 1) { // len == 1: one UTF-16 unit whatever the byte
            uint64_t hib = 0;
            const uint32_t s0 = q - len;
            const uint64_t a = R.sbase + s0;
            if (a + len + 8 <= R.rend || (R.rend == R.send && a + len <= R.rend)) {
              for (uint32_t k = 0; k < len; k += 8) {
                const uint32_t n8 = len - k < 8 ? len - k : 8;
                hib |= ring_read8(row, (uint32_t)(a + k - R.rb)) & (n8 == 8 ? ~0ull : ((1ull << (8 * n8)) - 1));
              }
            } else { // payload past the ring: read it from HBM (the lane refills after it)
              for (uint32_t k = 0; k < len; k++) hib |= up[s0 + k];
              wait = true;
            }
            if (hib & 0x8080808080808080ull) R.fail = F_BAIL; // non-ASCII: UTF-16 length / split checks
          }
        }
        if (!R.fail && reenc) R.fail = F_BAIL; // re-encoded sizes: general planner
        if (!R.fail) {
          const uint32_t bpos = pos, blen = q - pos;
          pos = q;
          if (kind == BK_ITEM && len == 0) { // Item::new -> None: dropped
            if (kb != 0xFFFFFFFFu) pure = 0;
          } else if ((uint64_t)clock + len > 0xFFFFFFFFull) {
            R.fail = F_BAIL;
          } else {
            nstored++;
            lkind = kind;
            lclock = clock;
            llen = len;
            if (DIFF) {
              if (!found) {
                if (kind != BK_SKIP && clock + len > remote) {
                  found = 1;
                  const uint32_t off = remote > clock ? remote - clock : 0;
                  uint32_t sz;
                  if (off == 0) {
                    sz = blen;
                  } else if (kind != BK_ITEM) {
                    sz = 1 + varlen(len - off);
                  } else {
                    // ItemSlice::encode with an offset (emit_block): origin (client, clock + off - 1)
                    // synthesised, right origin copied (canonical here), no parent info, content
                    // sliced (ASCII string: byte offset = UTF-16 offset)
                    const uint32_t rest = len - off;
                    sz = 1 + varlen(client) + varlen(clock + off - 1) + rbytes + varlen(rest) +
                         ((info & 15) == 4 ? rest : 0u);
                  }
                  uint32_t *sr = cl + CLW * e;
                  sr[6] = bpos;
                  sr[7] = clock;
                  sr[8] = len;
                  sr[9] = off;
                  sr[11] = sz;
                  if (off == 0) {
                    sr[14] = 1;
                  } else if (kind == BK_ITEM) { // OP_SLICE: right origin bytes, ref, parent_sub flag
                    const uint32_t has_ps = (info & 0xE0) == 0x20 ? 1u : 0u;
                    sr[12] = ropos;
                    sr[13] = rbytes | ((info & 15) << 8) | (has_ps << 12) | ((pos - ropos) << 16);
                    sr[14] = 2;
                  }
                  count = 1;
                  kb = pos;
                }
              } else {
                if (kb == 0xFFFFFFFFu) kb = bpos;
                count++;
                ssize += blen;
              }
            }
            clock += len;
          }
          if (!R.fail && ++j == nb) sec_end = true;
        }
      } else if (st == R_SEC) {
        // ---- section header: blocks count, client, first clock
        nb = f0;
        client = f1;
        clock = f2;
        if (!R.fail) {
          pos = q;
          uint32_t f = 0;
          while (f < nclients && ct.keys[f] != client) f++;
          if (f == nclients) { // entry(..).or_default (the table itself is built after the walk)
            nclients++;
            ct.keys[f] = client;
            uint32_t *sr = cl + CLW * f;
            for (uint32_t k = 0; k < CLW; k++) sr[k] = 0;
            if (DIFF) {
              const uint32_t *svt = scr + L.sq;
              uint32_t rc = 0;
              for (uint32_t k = 0; k < nsv; k++)
                if (svt[2 * k] == client) rc = svt[2 * k + 1];
              sr[4] = rc;
            }
          }
          e = f;
          const uint32_t *sr = cl + CLW * e;
          nstored = sr[0];
          lkind = sr[1];
          lclock = sr[2];
          llen = sr[3];
          remote = sr[4];
          found = sr[5];
          count = sr[10];
          if (((uint64_t)nstored + nb) * 32ull > ALLOC_LIMIT || nsec >= cap.C) R.fail = F_BAIL;
          kb = 0xFFFFFFFFu;
          pure = 1;
          ssize = 0;
          j = 0;
          if (nb) st = R_BLOCK;
          else sec_end = true;
        }
      } else if (st == R_DRANGE) {
        // ---- one DeleteSet range (start, len)
        const uint32_t rs = f0, rl = f1;
        if (!R.fail && (uint64_t)rs + rl > 0xFFFFFFFFull) R.fail = F_BAIL;
        if (!R.fail) {
          pos = q;
          dcanon &= (ncan & 3) == 0;
          if (kr > 0 && rs < prev_e) dsq = false;
          prev_e = rs + rl;
          dsz += varlen(rs) + varlen(rl);
          if (++kr == nr) entry_end = true;
        }
      } else if (st == R_DENT) {
        // ---- DeleteSet entry header: client, range count
        dclient = f0;
        nr = f1;
        if (!R.fail) {
          pos = q;
          cpos = p1;
          dcanon = (ncan & 2) == 0;
          dsq = true;
          prev_e = 0;
          dsz = varlen(nr);
          kr = 0;
          if (nr) st = R_DRANGE;
          else entry_end = true;
        }
      } else if (st == R_NCL) {
        ncl = f0;
        if (!R.fail && ncl > cap.C) R.fail = F_BAIL;
        if (!R.fail) {
          pos = q;
          st = ncl ? R_SEC : R_NDS;
        }
      } else { // R_NDS
        nds = f0;
        if (!R.fail && DIFF && nds > cap.E) R.fail = F_BAIL;
        if (!R.fail) {
          pos = q;
          ids = 0;
          st = nds ? R_DENT : R_DONE;
        }
      }
      if (R.fail == F_SHORT) { // nothing consumed: the item is read again after the refill
        wait = true;
        continue;
      }
      if (R.fail) {
        bail = true;
        active = false;
        continue;
      }
      if (sec_end) {
        if (kb == 0xFFFFFFFFu) kb = pos;
        uint32_t *sr = sec + SECW * nsec++;
        sr[0] = e;
        sr[1] = kb;
        sr[2] = pos;
        sr[3] = pure;
        sr[4] = ssize;
        uint32_t *cr = cl + CLW * e;
        cr[0] = nstored;
        cr[1] = lkind | 0x100;
        cr[2] = lclock;
        cr[3] = llen;
        cr[5] = found;
        cr[10] = count;
        st = ++isec < ncl ? R_SEC : R_NDS;
      }
      if (entry_end) {
        if (DIFF) {
          if (!dsq) { // squash of a clone: general planner
            bail = true;
            active = false;
            continue;
          }
          uint32_t *r = de + DEW * ids;
          r[0] = dclient;
          r[1] = cpos;
          r[2] = pos;
          r[3] = nr;
          r[4] = 1u | (dcanon ? 2u : 0u);
          r[7] = varlen(dclient) + dsz;
        }
        st = ++ids < nds ? R_DENT : R_DONE;
      }
      if (st == R_DONE) active = false;
    }
    if (ps.stamps) t_stp += __builtin_amdgcn_s_memtime() - tq;
  }
  const uint64_t tf0 = ps.stamps ? __builtin_amdgcn_s_memtime() : 0;
  if (d >= b.n_docs) return;
  if (!bail && st == R_DONE) {
    if (ncl && !ct.reserve(ncl, scr + L.ct_tmp)) bail = true;
    for (uint32_t f = 0; f < nclients && !bail; f++) {
      if (!ct.reserve(1, scr + L.ct_tmp)) bail = true;
      else ct.place(ct.keys[f], f);
    }
    if (DIFF) {
      for (uint32_t i = 0; i < nds && !bail; i++) {
        const uint32_t dc = de[DEW * i];
        if (!dt.reserve(1, scr + L.dt_tmp)) {
          bail = true;
          break;
        }
        const int f = dt.find(dc);
        if (f >= 0) { // replaced in place: the slot now names entry i
          for (uint32_t s = 0; s < dt.buckets; s++)
            if (dt.slot[s] == (uint32_t)f + 1) dt.slot[s] = i + 1;
          dt.keys[i] = dc;
        } else {
          dt.place(dc, i);
        }
      }
    }
    if (!bail) {
      uint64_t sz = 0;
      const uint32_t stt = plan_finish<DIFF>(scr, L, cap, ct, nsec, dt, false, 0u, sz);
      if (stt == PLAN_OVF) {
        bail = true;
      } else {
        if (b.frame && !stt) sz += 2 + varlen(sz); // y-sync message framing
        ps.big[d] = 0;
        ps.status[d] = (uint8_t)stt;
        ps.size[d] = stt ? 0 : sz;
      }
    }
  }
  if (bail) ps.big[d] = PLAN_REDO;
  if (ps.stamps) {
    uint64_t *o = ps.stamps + (size_t)d * 16;
    o[0] = t_ref;
    o[1] = t_stp;
    o[2] = __builtin_amdgcn_s_memtime() - tf0;
    o[3] = n_ref;
    o[4] = n_stp;
    o[5] = un;
    o[7] = 0xD1FF;
  }
}

template <bool DIFF>
__global__ void __launch_bounds__(64) k_plan(DiffBatch b, PlanScratch ps, int pass) {
  ym_set_grammar(b.v1x);
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= b.n_docs) return;
  if (pass == 1 && !ps.big[d]) return;
  if (pass == 0 && ps.big[d] != PLAN_REDO) return; // planned by k_plan_ring
  if (b.ls_done && b.ls_done[d]) return;
  if (b.pre_status && b.pre_status[d]) { // e.g. a y-sync message that is not SyncStep1
    ps.big[d] = 0;
    ps.status[d] = b.pre_status[d];
    ps.size[d] = 0;
    return;
  }
  const uint64_t o0 = b.upd_off[d], o1 = b.upd_off[d + 1];
  const uint8_t *up = b.bytes + o0;
  const uint32_t un = (uint32_t)(o1 - o0);
  const uint8_t *svp = nullptr;
  uint32_t svn = 0;
  if (DIFF) {
    svp = b.sv + b.sv_off[d];
    svn = (uint32_t)((b.sv_end ? b.sv_end[d] : b.sv_off[d + 1]) - b.sv_off[d]);
  }
  uint32_t *scr;
  PlanCaps cap;
  if (pass == 0) {
    cap = small_caps();
    scr = ps.small + (size_t)d * ps.small_words;
  } else {
    cap = big_caps(un);
    scr = ps.bigscr + ps.big_off[d];
  }
  uint64_t sz = 0;
  uint32_t st = plan_doc<DIFF>(up, un, svp, svn, scr, cap, sz);
  if (st == PLAN_OVF && pass == 1) st = validate_doc<DIFF>(up, un, svp, svn);
  if (st == PLAN_OVF) {
    // only the small pass can overflow (big capacities hold every decodable update)
    ps.big[d] = pass == 0 ? 1 : 0;
    ps.status[d] = pass == 0 ? 0 : E_OTHER;
    ps.size[d] = 0;
    if (pass == 0) atomicAdd(ps.n_big, 1u);
    return;
  }
  if (pass == 0) ps.big[d] = 0;
  // y-sync message: [MSG_SYNC, SyncStep2 | SyncStep1, varbuf(payload)] (protocol.rs:219-233)
  if (b.frame && !st) sz += 2 + varlen(sz);
  ps.status[d] = (uint8_t)st;
  ps.size[d] = st ? 0 : sz;
}

// y-sync client message -> state vector slice (Message::decode + SyncMessage::decode,
// yrs/src/sync/protocol.rs:179-203, 245-272; tags are read_var::<u8>)
__global__ void k_sync_parse(const uint8_t *msg, const uint64_t *msg_off, uint32_t n, uint64_t *sv_off,
                             uint64_t *sv_end, uint8_t *status) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  Cur c{msg + msg_off[d], (uint32_t)(msg_off[d + 1] - msg_off[d]), 0};
  bool cn;
  uint32_t tag = 0, sub = 0, len = 0;
  int e = rd_var_u32(c, tag, cn);
  if (!e && tag > 255) e = E_VARINT;
  if (!e && tag != 0) e = E_UNSUPPORTED; // awareness / auth / query / custom: not update algebra
  if (!e) e = rd_var_u32(c, sub, cn);
  if (!e && sub > 255) e = E_VARINT;
  if (!e && (sub == 1 || sub == 2)) e = E_UNSUPPORTED; // SyncStep2 / Update: applied, not answered
  if (!e && sub != 0) e = E_UNEXPECTED;
  if (!e) e = rd_var_u32(c, len, cn);
  if (!e && len > c.n - c.i) e = E_EOS;
  sv_off[d] = msg_off[d] + c.i;
  sv_end[d] = e ? msg_off[d] + c.i : msg_off[d] + c.i + len;
  status[d] = (uint8_t)e;
}
void launch_sync_parse(const uint8_t *msg, const uint64_t *msg_off, uint32_t n, uint64_t *sv_off, uint64_t *sv_end,
                       uint8_t *status, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_sync_parse, dim3((n + 255) / 256), dim3(256), 0, s, msg, msg_off, n, sv_off, sv_end, status);
}

__global__ void k_big_need(const uint64_t *upd_off, const uint8_t *big, uint32_t n, uint64_t *need) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  need[d] = big[d] ? (plan_big_words(upd_off[d + 1] - upd_off[d]) + 1) & ~1ull : 0;
}

// ------------------------------------------------------------------ executor
template <class W> __device__ __forceinline__ void walk_emit(const uint8_t *up, uint32_t un, uint32_t kb,
                                                             uint32_t ke, uint32_t client, W &w) {
  WCur c;
  wc_init(c, up, un);
  c.i = kb;
  while (c.i < ke) {
    const uint32_t bpos = c.i;
    BlockInfo bi;
    if (wparse_block(c, bi)) return;
    if (bi.kind == BK_ITEM && bi.len == 0) continue;
    if (!bi.reenc && !bi.enc_panic) {
      for (uint32_t q = bpos; q < c.i; q++) w.u8((uint8_t)wc_byte(c, q));
    } else {
      emit_block(up, un, bpos, client, 0, bi.len, 0, w);
    }
  }
}

// One wavefront copies len bytes (any alignments): byte stores up to the first 16-byte
// aligned destination address, then per lane 16-byte aligned stores assembled from the
// source dwords with v_alignbyte (every dword read holds at least one source byte, so no
// read leaves the source's pages), then the byte tail.
__device__ __forceinline__ void wave_copy(uint8_t *dst, const uint8_t *src, uint32_t len, uint32_t lane) {
  uint32_t h = (uint32_t)(-(uintptr_t)dst) & 15u;
  if (len < 64) h = len;
  if (lane < h) dst[lane] = src[lane];
  if (h == len) return;
  const uint32_t n16 = (len - h) >> 4;
  const uint8_t *s = src + h;
  uint4 *d = (uint4 *)(dst + h);
  const uint32_t sh = (uint32_t)(uintptr_t)s & 3u;
  const uint32_t *sa = (const uint32_t *)((uintptr_t)s & ~(uintptr_t)3);
  for (uint32_t k = lane; k < n16; k += 64) {
    const uint32_t *x = sa + 4 * k;
    const uint32_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3], x4 = sh ? x[4] : 0u;
    uint4 v;
    v.x = __builtin_amdgcn_alignbyte(x1, x0, sh);
    v.y = __builtin_amdgcn_alignbyte(x2, x1, sh);
    v.z = __builtin_amdgcn_alignbyte(x3, x2, sh);
    v.w = __builtin_amdgcn_alignbyte(x4, x3, sh);
    d[k] = v;
  }
  const uint32_t done = h + 16 * n16;
  if (lane < len - done) dst[done + lane] = src[done + lane];
}

// The op list of document d (small or length-sized plan scratch)
__device__ __forceinline__ const uint32_t *plan_ops(const DiffBatch &b, const PlanScratch &ps, uint32_t d, uint32_t un,
                                                    const uint32_t *&scr, PlanLayout &L) {
  if (ps.big[d]) {
    L = plan_layout(big_caps(un));
    scr = ps.bigscr + ps.big_off[d];
  } else {
    L = plan_layout(small_caps());
    scr = ps.small + (size_t)d * ps.small_words;
  }
  return scr + L.ops;
}

// Hot executor: one wavefront per document.  Wave scan of the op sizes (offsets stored in
// op word 7), the y-sync header, header varints and ASCII / Deleted slices one lane per op,
// verbatim ranges (most of the output) by the whole wave with 16-byte stores.  The re-encode
// ops (OP_EMIT / OP_WALK / OP_DSQ / OP_DSS: general-planner shapes) are k_exec_cold's, so
// this kernel keeps a small register footprint (no emit_block call).
__global__ void __launch_bounds__(256) k_exec(DiffBatch b, PlanScratch ps, const uint64_t *out_off, uint8_t *out) {
  ym_set_grammar(b.v1x);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t d = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (d >= b.n_docs) return;
  if (ps.status[d] || ps.size[d] == 0 || (b.ls_done && b.ls_done[d])) return;
  const uint64_t o0 = b.upd_off[d], o1 = b.upd_off[d + 1];
  const uint8_t *up = b.bytes + o0;
  const uint32_t un = (uint32_t)(o1 - o0);
  const uint32_t *scr;
  PlanLayout L;
  uint32_t *ops = (uint32_t *)plan_ops(b, ps, d, un, scr, L);
  const uint32_t nops = scr[0];
  uint8_t *dst = out + out_off[d];
  // op offsets: wave-wide exclusive scan of the sizes (acc = the unframed payload size)
  uint32_t acc = 0;
  for (uint32_t r = 0; r < nops; r += 64) {
    const uint32_t k = r + lane;
    const uint32_t sz = k < nops ? ops[OPW * k + 1] : 0;
    uint32_t x = sz;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (k < nops) ops[OPW * k + 7] = acc + x - sz;
    acc += __shfl(x, 63, 64);
  }
  if (b.frame) { // y-sync header [MSG_SYNC, step tag, varbuf length]
    const uint32_t hl = 2 + varlen(acc);
    if (lane == 0) {
      Writer w{dst, 0};
      w.u8(0);
      w.u8(b.frame == 1 ? 1 : 0);
      w_var(w, acc);
    }
    dst += hl;
  }
  for (uint32_t k = lane; k < nops; k += 64) {
    const uint32_t *o = ops + OPW * k;
    Writer w{dst + o[7], 0};
    if (o[0] == OP_VARS) {
      w_var(w, o[3]);
      if (o[2] > 1) w_var(w, o[4]);
      if (o[2] > 2) w_var(w, o[5]);
    } else if (o[0] == OP_SLICE) {
      // ItemSlice::encode with an offset (slice.rs:199-251 as emit_block does it): origin
      // (client, clock + off - 1), the right origin's bytes, no parent info; content: the
      // remaining length, and for a String the payload's last `rest` bytes (ASCII)
      const uint32_t ro = o[4], pk = o[5], rest = o[6];
      const uint32_t rbytes = pk & 0xFF, ref = (pk >> 8) & 15, ps_flag = (pk >> 12) & 1, bend = ro + (pk >> 16);
      w.u8((uint8_t)(0x80 | (rbytes ? 0x40 : 0) | (ps_flag ? 0x20 : 0) | ref));
      w_var(w, o[2]);
      w_var(w, o[3]);
      for (uint32_t q = 0; q < rbytes; q++) w.u8(up[ro + q]);
      w_var(w, rest);
      if (ref == 4)
        for (uint32_t q = 0; q < rest; q++) w.u8(up[bend - rest + q]);
    }
  }
  // verbatim ranges: all lanes, 16-byte aligned stores
  for (uint32_t k = 0; k < nops; k++) {
    const uint32_t *o = ops + OPW * k;
    if (o[0] != OP_COPY) continue;
    wave_copy(dst + o[7], up + o[2], o[1], lane);
  }
}

// Cold executor (after k_exec, whose scan stored the op offsets): one lane per document
// writes the re-encode ops — emit_block with an offset, a section walked block by block,
// squashed or re-encoded DeleteSet ranges.
__global__ void __launch_bounds__(64) k_exec_cold(DiffBatch b, PlanScratch ps, const uint64_t *out_off, uint8_t *out) {
  ym_set_grammar(b.v1x);
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= b.n_docs) return;
  if (ps.status[d] || ps.size[d] == 0 || (b.ls_done && b.ls_done[d])) return;
  const uint64_t o0 = b.upd_off[d], o1 = b.upd_off[d + 1];
  const uint8_t *up = b.bytes + o0;
  const uint32_t un = (uint32_t)(o1 - o0);
  const uint32_t *scr;
  PlanLayout L;
  const uint32_t *ops = plan_ops(b, ps, d, un, scr, L);
  const uint32_t nops = scr[0];
  bool any = false;
  uint32_t acc = 0;
  for (uint32_t k = 0; k < nops; k++) {
    const uint32_t kind = ops[OPW * k];
    any |= kind == OP_EMIT || kind == OP_WALK || kind == OP_DSQ || kind == OP_DSS;
    acc += ops[OPW * k + 1];
  }
  if (!any) return;
  uint8_t *dst = out + out_off[d] + (b.frame ? 2 + varlen(acc) : 0);
  for (uint32_t k = 0; k < nops; k++) {
    const uint32_t *o = ops + OPW * k;
    Writer w{dst + o[7], 0};
    switch (o[0]) {
    case OP_EMIT: emit_block(up, un, o[2], o[6], o[3], o[4], o[5], w); break;
    case OP_WALK: walk_emit(up, un, o[2], o[3], o[6], w); break;
    case OP_DSQ: {
      const uint32_t *v = scr + L.sq + 2 * o[2];
      w_var(w, o[3]);
      for (uint32_t q = 0; q < o[3]; q++) {
        w_var(w, v[2 * q]);
        w_var(w, v[2 * q + 1] - v[2 * q]);
      }
      break;
    }
    case OP_DSS: {
      WCur c;
      wc_init(c, up, un);
      c.i = o[2];
      bool cn;
      uint32_t n, s0, ln;
      wc_var_u32(c, n, cn);
      w_var(w, n);
      for (uint32_t q = 0; q < n; q++) {
        wc_var_u32(c, s0, cn);
        wc_var_u32(c, ln, cn);
        w_var(w, s0);
        w_var(w, ln);
      }
      break;
    }
    default: break;
    }
  }
}

void launch_plan(bool diff, int pass, const DiffBatch &b, const PlanScratch &ps, hipStream_t s) {
  if (!b.n_docs) return;
  if (pass == 0 && ps.planner == 1) { // common shapes, the ring planner (env YMERGE_PLANNER=ring)
    dim3 gr((b.n_docs + RING_NT - 1) / RING_NT), tr(RING_NT);
    if (diff)
      hipLaunchKernelGGL(k_plan_ring<true>, gr, tr, 0, s, b, ps);
    else
      hipLaunchKernelGGL(k_plan_ring<false>, gr, tr, 0, s, b, ps);
  } else if (pass == 0 && ps.planner == 2) { // every document on a wavefront (env YMERGE_PLANNER=wave)
    PlanScratch pw = ps;
    pw.wave_list = nullptr;
    dim3 gr((b.n_docs + PW_WPB - 1) / PW_WPB), tr(64 * PW_WPB);
    if (diff)
      hipLaunchKernelGGL(k_plan_wave<true>, gr, tr, 0, s, b, pw);
    else
      hipLaunchKernelGGL(k_plan_wave<false>, gr, tr, 0, s, b, pw);
  } else if (pass == 0) { // lane per document; documents of >= PW_MIN bytes on a wavefront each
    dim3 gr((b.n_docs + RING_NT - 1) / RING_NT), tr(RING_NT), gw(256), tw(64 * PW_WPB);
    if (diff) {
      hipLaunchKernelGGL(k_plan_lane<true>, gr, tr, 0, s, b, ps);
      hipLaunchKernelGGL(k_plan_wave<true>, gw, tw, 0, s, b, ps);
    } else {
      hipLaunchKernelGGL(k_plan_lane<false>, gr, tr, 0, s, b, ps);
      hipLaunchKernelGGL(k_plan_wave<false>, gw, tw, 0, s, b, ps);
    }
  }
  // the documents the common-shape planners left (ps.big = PLAN_REDO)
  dim3 g((b.n_docs + 63) / 64), t(64);
  if (diff)
    hipLaunchKernelGGL(k_plan<true>, g, t, 0, s, b, ps, pass);
  else
    hipLaunchKernelGGL(k_plan<false>, g, t, 0, s, b, ps, pass);
}
void launch_big_need(const uint64_t *upd_off, const uint8_t *big, uint32_t n, uint64_t *need, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_big_need, dim3((n + 255) / 256), dim3(256), 0, s, upd_off, big, n, need);
}
void launch_exec(const DiffBatch &b, const PlanScratch &ps, const uint64_t *out_off, uint8_t *out, hipStream_t s) {
  if (!b.n_docs) return;
  hipLaunchKernelGGL(k_exec, dim3((b.n_docs + 3) / 4), dim3(256), 0, s, b, ps, out_off, out);
  hipLaunchKernelGGL(k_exec_cold, dim3((b.n_docs + 63) / 64), dim3(64), 0, s, b, ps, out_off, out);
}

} // namespace ym
