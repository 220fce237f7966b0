// ymerge_big.hip — merge_updates_v1 for documents above the fast path's LDS capacities.
//
// The fast path (ymerge_fast.hip) keeps a whole document in LDS: at most 1024 blocks,
// 512 DeleteSet entries / ranges, 64 distinct DeleteSet clients.  Documents beyond
// that (Zipf-tail tenants of C3, long per-op logs such as the automerge-paper trace,
// delete-heavy logs) run here with the same semantics, one 512-lane workgroup per
// document, the SoA block / DeleteSet tables in HBM scratch and every phase a loop
// over tiles of one element per lane with a carry between tiles:
//   k_big_count  per document: counts (blocks, entries, ranges) from the k_decode
//                records, first decode error, scratch words
//   k_big_merge  gather records -> sort blocks by (client desc, clock asc, input order)
//                (skipped when already ordered; else LDS bitonic chunks + stable merge
//                passes) -> classify (segmented max-scan of block ends: keep / Skip gap /
//                violation, duplicate check) -> sizes + offsets -> write (LDS-staged
//                tiles) -> DeleteSet: distinct clients + first occurrence (LDS hash),
//                hashbrown iteration order, ranges sorted by (client, start), segmented
//                union, write.
// Overlapping documents (partial overlaps, same-clock blocks that differ — snapshot +
// pending-log merges) switch to the run order of the yrs loop (big_run_order below) and
// write the overlapping blocks spliced; the exact engine (path = 1) keeps only the
// shapes that order does not cover (see big_run_order).
// Reference semantics: yrs/src/update.rs:537-704 (merge), :490-535 (encode),
// yrs/src/id_set.rs:129-164, 385-410 (DeleteSet union and order).
#include "yblock.h"
#include "ycopy.h"

namespace ym {

constexpr uint32_t BIG_DCAP = 1024;   // distinct DeleteSet clients per document
constexpr uint32_t BIG_DTAB = 2048;   // LDS hash slots for them (u64)
constexpr uint32_t BIG_CHUNK = 2048;  // LDS bitonic chunk of the sort (key u64 + value u32)
constexpr uint32_t BIG_LU_LDS = 8192;
constexpr uint32_t BIG_COOP = 64;
#ifndef YM_DS_PACKED
#define YM_DS_PACKED 1
#endif
constexpr bool BIG_DS_PACKED = YM_DS_PACKED; // DeleteSet range sort on packed keys (few clients)      // records of one update from which the gather copies them cooperatively // overlap mode: updates / runs whose last-rank histogram stays in LDS
// LDS union region (phase-local): sort chunk (24 KB) / output stage / DeleteSet tables:
//   [0, 16K) client hash table  [16K, 44K) 7 per-client arrays  [44K, 68K) sort chunk / slots
constexpr uint32_t BIG_OFF_DARR = 8 * BIG_DTAB, BIG_OFF_SCR = BIG_OFF_DARR + 7 * 4 * BIG_DCAP;
constexpr uint32_t BIG_UNION = BIG_OFF_SCR + 12 * BIG_CHUNK;

struct BigMem {
  uint32_t *bc, *bk, *bl, *bp, *bm; // [NB] blocks in input order
  uint64_t *k0, *k1;                // [M] sort keys (ping-pong)
  uint32_t *v0, *v1;                // [M] sort values
  uint32_t *fE, *fF, *sseg;         // [NB] per sorted position: running end, flags; per client segment counts
  uint32_t *fO;                     // [NB] per sorted position: splice offset (overlap mode)
  uint32_t *ec, *et;                // [NE] DeleteSet entries
  uint32_t *rs, *re, *ri;           // [NR] DeleteSet ranges
  uint32_t *chead, *cend, *coff, *cpre; // [NR + 1] union of sorted live ranges
  // overlap mode: per block update / run, sorted position -> block; per run (<= NB runs):
  // first block, blocks, client, start, update, first-block kind, previous run of its
  // update, rank, rank -> run (two buffers), first sorted block position; per update: last rank
  uint32_t *bu, *rr, *sord;
  uint32_t *Rb, *Rn, *Rc, *Rs, *Ru, *Rk, *Rp, *Rpos, *Rord, *Rord2, *Roff;
  uint32_t *lu;
};
__host__ __device__ inline uint64_t big_words(uint32_t NB, uint32_t NE, uint32_t NR, uint32_t U) {
  const uint64_t M = (uint64_t)(NB > NR ? NB : NR) + 2;
  return 4 * M + 2 * M + 9ull * NB + 2ull * NE + 3ull * NR + 4ull * (NR + 2) + 14ull * (NB + 2) + U + 96;
}
__device__ inline BigMem big_carve(uint32_t *w, uint32_t NB, uint32_t NE, uint32_t NR, uint32_t U) {
  BigMem m;
  const uint64_t M = (uint64_t)(NB > NR ? NB : NR) + 2;
  uint64_t o = 0;
  auto take = [&](uint64_t k) {
    uint32_t *p = w + o;
    o += (k + 1) & ~1ull; // keep 8-byte alignment
    return p;
  };
  m.k0 = (uint64_t *)take(2 * M);
  m.k1 = (uint64_t *)take(2 * M);
  m.v0 = take(M);
  m.v1 = take(M);
  m.bc = take(NB);
  m.bk = take(NB);
  m.bl = take(NB);
  m.bp = take(NB);
  m.bm = take(NB);
  m.fE = take(NB);
  m.fF = take(NB);
  m.sseg = take(NB);
  m.ec = take(NE);
  m.et = take(NE);
  m.rs = take(NR);
  m.re = take(NR);
  m.ri = take(NR);
  m.chead = take(NR + 2);
  m.cend = take(NR + 2);
  m.coff = take(NR + 2);
  m.cpre = take(NR + 2);
  m.fO = take(NB);
  m.bu = take(NB);
  m.rr = take(NB);
  m.sord = take(NB);
  uint32_t **ra[11] = {&m.Rb, &m.Rn, &m.Rc, &m.Rs, &m.Ru, &m.Rk, &m.Rp, &m.Rpos, &m.Rord, &m.Rord2, &m.Roff};
  for (int i = 0; i < 11; i++) *ra[i] = take(NB + 1);
  m.lu = take(U);
  return m;
}
// The tables' addresses are per document, so wave-uniform: pinned to scalar registers (the
// compiler otherwise kept several of them as VGPR pairs, a large part of the kernel's spills)
template <class T> __device__ __forceinline__ T *uni_ptr(T *p) {
  const uint64_t x = (uint64_t)p;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return (T *)(((uint64_t)hi << 32) | lo);
}
__device__ inline void big_uniform(BigMem &m) {
  uint32_t **p32[] = {&m.bc, &m.bk, &m.bl, &m.bp, &m.bm, &m.v0, &m.v1, &m.fE, &m.fF, &m.sseg, &m.fO, &m.ec, &m.et,
                      &m.rs, &m.re, &m.ri, &m.chead, &m.cend, &m.coff, &m.cpre, &m.bu, &m.rr, &m.sord, &m.Rb, &m.Rn,
                      &m.Rc, &m.Rs, &m.Ru, &m.Rk, &m.Rp, &m.Rpos, &m.Rord, &m.Rord2, &m.Roff, &m.lu};
#pragma unroll
  for (uint32_t i = 0; i < sizeof(p32) / sizeof(p32[0]); i++) *p32[i] = uni_ptr(*p32[i]);
  m.k0 = uni_ptr(m.k0);
  m.k1 = uni_ptr(m.k1);
}

// ------------------------------------------------------------------ k_big_count
// One workgroup per document with path == 2 (handed over by k_fast_merge for capacity):
// counts, first decode error in update order (yrs/src/alt.rs:21-25), scratch words.
template <int NT>
__global__ void __launch_bounds__(NT) k_big_count(BatchIn b, uint8_t *path, uint8_t *status, uint64_t *out_start,
                                                  uint64_t *out_len, uint32_t *counts, uint64_t *need,
                                                  uint32_t *n_big, uint32_t *npath, const uint32_t *list) {
  ym_set_grammar(b.v1x);
  const uint32_t d = list[blockIdx.x];
  if (d >= b.n_docs) return;
  const uint32_t t = threadIdx.x;
  if (path[d] != 2) {
    if (t == 0) need[d] = 0;
    return;
  }
  __shared__ unsigned long long s_err, s_nb, s_ne, s_nr;
  __shared__ uint32_t s_flags;
  if (t == 0) {
    s_err = ~0ull;
    s_nb = s_ne = s_nr = 0;
    s_flags = 0;
  }
  __syncthreads();
  const uint64_t u0 = b.doc_upd[d], u1 = b.doc_upd[d + 1];
  const uint32_t U = (uint32_t)(u1 - u0);
  const uint64_t B0 = b.upd_off[u0];
  uint64_t nb = 0, ne = 0, nr = 0;
  uint32_t flags = 0;
  for (uint32_t i = t; i < U; i += NT) {
    const uint64_t a0 = b.upd_off[u0 + i], a1 = b.upd_off[u0 + i + 1];
    const uint32_t ulen = (uint32_t)(a1 - a0);
    const uint2 *rp = (const uint2 *)(b.rec + (size_t)(u0 + i) * REC_WORDS);
    const uint2 x0 = rp[0], x1 = rp[1];
    uint32_t w0 = x0.x, w1 = x0.y, w2 = x1.x, w3 = x1.y, w4 = 0, w5 = 0;
    if (w0 & REC_SLOW) {
      RegSink s;
      s.nb = s.ne = s.nr = 0;
      s.unsupported = s.big_ds = false;
      s.ubase = 0;
      WCur c;
      wc_init(c, b.bytes + a0, ulen);
      const int es = smwalk_update(c, s);
      rec_pack(s, es, w0, w1, w2, w3, w4, w5);
    }
    const uint32_t e = w0 & 0xFF, shape = (w0 >> 10) & 3;
    if (e) atomicMin(&s_err, ((unsigned long long)i << 8) | e);
    if (w0 & REC_BIGDS) flags |= 2;
    if (w0 & REC_ORDER) flags |= 16;
    if (ulen >= (1u << 24)) flags |= 8;
    if (!e) {
      if (shape == REC_BLOCK) nb += 1;
      else if (shape == REC_DS) {
        ne += 1;
        nr += (w0 >> 12) & 3;
      } else if (shape == REC_COMPLEX) {
        nb += w1;
        ne += w2;
        nr += w3;
      }
    }
  }
  atomicAdd(&s_nb, (unsigned long long)nb);
  atomicAdd(&s_ne, (unsigned long long)ne);
  atomicAdd(&s_nr, (unsigned long long)nr);
  if (flags) atomicOr(&s_flags, flags);
  __syncthreads();
  if (t != 0) return;
  const uint64_t slot = 2 * B0 + 64ull * d;
  need[d] = 0;
  if (s_err != ~0ull) { // the first failing update decides the document (yrs/src/alt.rs:21-25)
    status[d] = (uint8_t)(s_err & 0xFF);
    path[d] = 0;
    out_len[d] = 0;
    out_start[d] = slot;
    return;
  }
  // per-update DeleteSet tables beyond DS_SMALL entries, blocks over 16 MB, documents
  // whose offsets do not fit the 32-bit tables: exact engine
  if (s_flags || s_nb >= (1ull << 28) || s_ne >= (1ull << 28) || s_nr >= (1ull << 28) ||
      b.upd_off[u1] - B0 >= (1ull << 30)) {
    path[d] = 1;
    atomicAdd(&npath[1], 1u);
    return;
  }
  counts[4 * d + 1] = (uint32_t)s_nb;
  counts[4 * d + 2] = (uint32_t)s_ne;
  counts[4 * d + 3] = (uint32_t)s_nr;
  need[d] = (big_words((uint32_t)s_nb, (uint32_t)s_ne, (uint32_t)s_nr, U) + 1) & ~1ull;
  atomicAdd(n_big, 1u);
}

// ------------------------------------------------------------------ register bitonic
// Ascending sort of BIG_CHUNK (key u64, value u32) pairs by (key, value) held in registers,
// E = BIG_CHUNK / NT consecutive elements per lane: strides below E are exchanged inside the
// lane, strides below 64 E across the wavefront by lane shuffles, and only the strides of
// 64 E and more (6 of the 66 stages for NT = 512) go through LDS with two barriers each (the
// LDS-only bitonic paid a barrier on every stage).  Positions at or past n are padding
// (~0, ~0), sorted last; k / v hold the input and receive the first n results.
// KO: keys only (distinct keys, v unused): one 64-bit compare and no value moves per exchange
template <int NT, bool KO = false> __device__ void bitonic_reg(uint64_t *k, uint32_t *v, uint32_t n) {
  constexpr uint32_t E = BIG_CHUNK / NT;
  static_assert(E >= 1 && E * NT == BIG_CHUNK, "one chunk per workgroup");
  const uint32_t t = threadIdx.x;
  uint64_t x[E];
  uint32_t y[E];
#pragma unroll
  for (uint32_t r = 0; r < E; r++) {
    const uint32_t e = t * E + r;
    x[r] = e < n ? k[e] : ~0ull;
    y[r] = KO ? 0u : (e < n ? v[e] : 0xFFFFFFFFu);
  }
  // element e at the lower position of its pair keeps the minimum in an ascending block
  auto pick = [](uint64_t &a, uint32_t &av, uint64_t b, uint32_t bv, bool want_min) {
    const bool g = a > b || (!KO && a == b && av > bv);
    if (g == want_min) {
      a = b;
      av = bv;
    }
  };
  for (uint32_t size = 2; size <= BIG_CHUNK; size <<= 1) {
    for (uint32_t st = size >> 1; st > 0; st >>= 1) {
      if (st >= 64 * E) {
        __syncthreads();
#pragma unroll
        for (uint32_t r = 0; r < E; r++) {
          k[t * E + r] = x[r];
          if (!KO) v[t * E + r] = y[r];
        }
        __syncthreads();
        uint64_t px[E];
        uint32_t py[E];
#pragma unroll
        for (uint32_t r = 0; r < E; r++) {
          const uint32_t e = t * E + r;
          px[r] = k[e ^ st];
          py[r] = KO ? 0u : v[e ^ st];
        }
#pragma unroll
        for (uint32_t r = 0; r < E; r++) {
          const uint32_t e = t * E + r;
          pick(x[r], y[r], px[r], py[r], !(e & st) == !(e & size));
        }
      } else if (st >= E) {
        const int ls = (int)(st / E);
#pragma unroll
        for (uint32_t r = 0; r < E; r++) {
          const uint32_t e = t * E + r;
          const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x[r], ls, 64);
          const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x[r] >> 32), ls, 64);
          const uint32_t pv = KO ? 0u : (uint32_t)__shfl_xor((int)y[r], ls, 64);
          pick(x[r], y[r], ((uint64_t)hi << 32) | lo, pv, !(e & st) == !(e & size));
        }
      } else {
#pragma unroll
        for (uint32_t ss = 1; ss < E; ss <<= 1)
          if (ss == st) {
#pragma unroll
            for (uint32_t r = 0; r < E; r++)
              if (!(r & ss)) {
                const uint32_t e = t * E + r;
                const uint64_t a = x[r], b = x[r | ss];
                const uint32_t av = y[r], bv = y[r | ss];
                const bool g = a > b || (!KO && a == b && av > bv);
                if (g == !(e & size)) {
                  x[r] = b;
                  y[r] = bv;
                  x[r | ss] = a;
                  y[r | ss] = av;
                }
              }
          }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < E; r++) {
    const uint32_t e = t * E + r;
    if (e < n) {
      k[e] = x[r];
      if (!KO) v[e] = y[r];
    }
  }
  __syncthreads();
}

// ------------------------------------------------------------------ workgroup sort
// Stable sort of (key, value) pairs in HBM by key; values are distinct and ascending in
// input order.  Chunks of BIG_CHUNK pairs are bitonic-sorted in LDS by (key, value) —
// which equals the stable order — then bottom-up merge passes place every element at
// base + i + (rank in the partner run): left-run elements count partner keys < k,
// right-run elements count partner keys <= k (equal keys keep input order).
// Returns the buffer pair holding the result (0: k0/v0, 1: k1/v1).
// KO: keys only (distinct keys; v0 / v1 unused)
template <int NT, bool KO = false>
__device__ int wg_sort(uint64_t *k0, uint32_t *v0, uint64_t *k1, uint32_t *v1, uint32_t n, uint8_t *lds) {
  uint64_t *ck = (uint64_t *)lds;
  uint32_t *cv = (uint32_t *)(lds + 8 * BIG_CHUNK);
  const uint32_t CH = n < BIG_CHUNK ? pow2ceil(n < 2 ? 2 : n) : BIG_CHUNK; // chunk no larger than the input
  for (uint32_t c0 = 0; c0 < n; c0 += CH) {
    for (uint32_t j = threadIdx.x; j < CH; j += NT) {
      const uint32_t g = c0 + j;
      ck[j] = g < n ? k0[g] : ~0ull;
      if (!KO) cv[j] = g < n ? v0[g] : 0xFFFFFFFFu;
    }
    __syncthreads();
    bitonic_reg<NT, KO>(ck, cv, CH);
    for (uint32_t j = threadIdx.x; j < CH; j += NT) {
      const uint32_t g = c0 + j;
      if (g < n) {
        k0[g] = ck[j];
        if (!KO) v0[g] = cv[j];
      }
    }
    __syncthreads();
  }
  uint64_t *ka = k0, *kb = k1;
  uint32_t *va = v0, *vb = v1;
  int which = 0;
  // Merge passes.  The partner-run search runs over an LDS copy of every `stride`-th key
  // (BIG_CHUNK samples, the chunk area is free now) and finishes over HBM in log2(stride)
  // steps: a 4096-range DeleteSet (two chunks) merges with LDS reads only, instead of a
  // dependent chain of 11 HBM loads per element.
  uint64_t *smp = (uint64_t *)lds;
  uint32_t stride = 1;
  while ((n + stride - 1) / stride > BIG_CHUNK) stride <<= 1;
  for (uint32_t w = CH; w < n; w <<= 1) {
    const bool sampled = stride <= w; // runs start at multiples of w: samples align with them
    if (sampled) {
      for (uint32_t q = threadIdx.x; q * stride < n; q += NT) smp[q] = ka[q * stride];
      __syncthreads();
    }
    // four elements per lane per trip, each step's loads issued together (the chain per
    // element is key -> LDS samples -> log2(stride) HBM steps -> value)
    constexpr uint32_t MB = 4;
    for (uint32_t j0 = threadIdx.x; j0 < n; j0 += MB * NT) {
      uint64_t kj[MB];
      uint32_t lo[MB], hi[MB], b0[MB], base[MB];
      bool left[MB];
#pragma unroll
      for (uint32_t q = 0; q < MB; q++) {
        const uint32_t j = j0 + q * NT;
        kj[q] = j < n ? ka[j] : 0;
      }
#pragma unroll
      for (uint32_t q = 0; q < MB; q++) {
        const uint32_t j = j0 + q * NT < n ? j0 + q * NT : n - 1;
        const uint32_t run = j / w;
        left[q] = !(run & 1);
        base[q] = (left[q] ? run : run - 1) * w;
        uint32_t l = left[q] ? base[q] + w : base[q], h = left[q] ? base[q] + 2 * w : base[q] + w;
        if (l > n) l = n;
        if (h > n) h = n;
        b0[q] = l;
        if (sampled && l < h) {
          // samples q in [l / stride, ceil(h / stride)): the predicate holds on a prefix of
          // the run, so the count of true samples sn brackets the count: ((sn-1) stride, sn stride]
          uint32_t qa = l / stride, qb = (h + stride - 1) / stride;
          const uint32_t q0 = qa;
          while (qa < qb) {
            const uint32_t mid = (qa + qb) >> 1;
            const uint64_t km = smp[mid];
            if (left[q] ? (km < kj[q]) : (km <= kj[q])) qa = mid + 1;
            else qb = mid;
          }
          const uint32_t sn = qa - q0;
          if (sn == 0) {
            h = l;
          } else {
            const uint32_t nh = l + sn * stride;
            l = l + (sn - 1) * stride + 1;
            if (nh < h) h = nh;
          }
        }
        lo[q] = l;
        hi[q] = h;
      }
      // HBM steps in lockstep over the four searches
      for (;;) {
        bool any = false;
        uint64_t km[MB];
#pragma unroll
        for (uint32_t q = 0; q < MB; q++) {
          const bool act = lo[q] < hi[q];
          any |= act;
          km[q] = act ? ka[(lo[q] + hi[q]) >> 1] : 0;
        }
        if (!any) break;
#pragma unroll
        for (uint32_t q = 0; q < MB; q++) {
          if (lo[q] < hi[q]) {
            const uint32_t mid = (lo[q] + hi[q]) >> 1;
            if (left[q] ? (km[q] < kj[q]) : (km[q] <= kj[q])) lo[q] = mid + 1;
            else hi[q] = mid;
          }
        }
      }
      uint32_t vj[MB];
#pragma unroll
      for (uint32_t q = 0; q < MB; q++) {
        const uint32_t j = j0 + q * NT;
        vj[q] = !KO && j < n ? va[j] : 0;
      }
#pragma unroll
      for (uint32_t q = 0; q < MB; q++) {
        const uint32_t j = j0 + q * NT;
        if (j < n) {
          const uint32_t dst = base[q] + (j - (j / w) * w) + (lo[q] - b0[q]);
          kb[dst] = kj[q];
          if (!KO) vb[dst] = vj[q];
        }
      }
    }
    __syncthreads();
    uint64_t *tk = ka;
    ka = kb;
    kb = tk;
    uint32_t *tv = va;
    va = vb;
    vb = tv;
    which ^= 1;
  }
  return which;
}

// ------------------------------------------------------------------ overlap mode
// Can block (pos, clock length len) be written from offset `off` the way the exact engine
// writes a BlockCarrier::splice (update.rs:795-816, block.rs:1837-1879): GC, Deleted, JSON,
// Any, and Strings whose split keeps len - off UTF-16 units and re-encodes cleanly.  Other
// contents make yrs panic (ItemContent::splice -> None); those documents go to the exact
// engine, which reports it.
__device__ __noinline__ bool big_splice_ok(const uint8_t *p, uint32_t n, uint32_t pos, uint32_t len, uint32_t off) {
  Cur c{p, n, pos};
  uint8_t info;
  bool cn;
  uint32_t v;
  if (rd_u8(c, info)) return false;
  if (info == 0) return true;
  if (info & 0x80) {
    rd_var_u32(c, v, cn);
    rd_var_u32(c, v, cn);
  }
  if (info & 0x40) {
    rd_var_u32(c, v, cn);
    rd_var_u32(c, v, cn);
  }
  if ((info & 0xC0) == 0) {
    uint32_t pi;
    rd_var_u32(c, pi, cn);
    if (pi == 1) {
      rd_var_u32(c, v, cn);
      c.i += v;
    } else {
      rd_var_u32(c, v, cn);
      rd_var_u32(c, v, cn);
    }
    if (info & 0x20) {
      rd_var_u32(c, v, cn);
      c.i += v;
    }
  }
  const uint8_t ref = info & 15;
  if (ref == 1 || ref == 2 || ref == 8) return true;
  if (ref != 4) return false;
  if (rd_var_u32(c, v, cn) || c.i + v > n) return false;
  const uint8_t *str = p + c.i;
  uint32_t bo, bo2;
  if (str_split16(str, v, off, bo) || bo >= v) return false;
  if (str_len16(str + bo, v - bo) != len - off) return false;
  return str_split16(str + bo, v - bo, len - off, bo2) == 0;
}

// Order in which yrs' loop (update.rs:565-697) consumes the blocks of an overlapping
// document.  Each update's decoder yields its client sections in descending client order
// (IntoBlocks, update.rs:1030-1045); a "run" is a maximal contiguous stretch of one
// section.  Once a decoder is popped, the skip loop (:611-620) drops its covered blocks,
// the straddling block is spliced (:656-679) and the inner loop (:686-696) writes the rest
// of the run in the same iteration: runs are consumed whole, one per pop.  The live
// decoders are (re)sorted by their current run's (client desc, start asc); equal keys keep
// the deque order — the decoder popped most recently first, decoders never popped after
// them by input index — which is the heap order of the oracle (yrs_oracle.c
// merge_blocks).  So the runs are sorted by (client desc, start asc) and every tie group
// by (rank of the run's predecessor in its update desc, no predecessor last, update asc),
// refined until stable (the predecessor has a smaller key, so the refinement is a DAG
// walk).  Returns false (-> exact engine) for: a client with two runs in one update (a
// Skip inside a section, or a repeated section), a tie group above 256 runs or over 16
// refinement rounds, and an Item-vs-GC tie among the runs consumed while <= 20 decoders
// are live (Rust's insertion-sort regime).  On success m.sord[j] is the
// block at sorted position j (runs in order, blocks in run order).
template <int NT>
__device__ __noinline__ bool big_run_order(const BatchIn &b, uint64_t u0, uint32_t U, uint64_t B0, uint32_t NB,
                                           BigMem &m, uint32_t *ws, uint32_t *sc, uint8_t *lds, uint64_t *stp) {
  const uint32_t t = threadIdx.x;
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  auto mark = [&](uint32_t k) { // diagnostic builds only (stp = this document's stamps)
    if (stp) {
      __syncthreads();
      if (t == 0) stp[k] = __builtin_amdgcn_s_memtime();
    }
  };
  // 1 run heads and ids (m.bu: the update of every block, written by the gather)
  uint32_t NRun = 0;
  for (uint32_t base = 0; base < NB; base += NT) {
    const uint32_t j = base + t;
    bool h = false;
    if (j < NB)
      h = j == 0 || m.bu[j] != m.bu[j - 1] || m.bc[j] != m.bc[j - 1] || m.bk[j] != m.bk[j - 1] + m.bl[j - 1];
    uint32_t T;
    const uint32_t pre = bscan_sum<NT>(h ? 1u : 0u, ws, T);
    if (j < NB) {
      const uint32_t r = NRun + pre + (h ? 1 : 0) - 1;
      m.rr[j] = r;
      if (h) {
        m.Rb[r] = j;
        m.Rc[r] = m.bc[j];
        m.Rs[r] = m.bk[j];
        m.Ru[r] = m.bu[j];
        m.Rk[r] = m.bm[j] & 3;
      }
    }
    NRun += T;
  }
  __syncthreads();
  for (uint32_t r = t; r < NRun; r += NT) m.Rn[r] = (r + 1 < NRun ? m.Rb[r + 1] : NB) - m.Rb[r];
  mark(6);
  // 2 predecessor of every run in its update's stream (clients descending): sort by
  //   (update, client desc); a repeated (update, client) -> exact engine
  uint32_t bad = 0;
  for (uint32_t r = t; r < NRun; r += NT) {
    m.k0[r] = ((uint64_t)m.Ru[r] << 32) | (uint32_t)~m.Rc[r];
    m.v0[r] = r;
  }
  __syncthreads();
  const uint32_t *pv = m.v0;
  {
    uint32_t uns = 0;
    for (uint32_t r = t; r + 1 < NRun; r += NT) uns |= m.k0[r] > m.k0[r + 1];
    if (__syncthreads_or(uns) && wg_sort<NT>(m.k0, m.v0, m.k1, m.v1, NRun, lds)) pv = m.v1;
  }
  const uint64_t *pk = pv == m.v0 ? m.k0 : m.k1;
  for (uint32_t j = t; j < NRun; j += NT) {
    const uint32_t r = pv[j];
    uint32_t pr = NONE;
    if (j > 0 && (pk[j] >> 32) == (pk[j - 1] >> 32)) {
      if (pk[j] == pk[j - 1]) bad = 1;
      pr = pv[j - 1];
    }
    m.Rp[r] = pr;
  }
  if (__syncthreads_or(bad)) return false;
  mark(13);
  // 3 runs by (client desc, start asc, run id): run ids ascend with the update index
  for (uint32_t r = t; r < NRun; r += NT) {
    m.k0[r] = ((uint64_t)(uint32_t)~m.Rc[r] << 32) | m.Rs[r];
    m.v0[r] = r;
  }
  __syncthreads();
  const uint32_t *ov = m.v0;
  {
    uint32_t uns = 0;
    for (uint32_t r = t; r + 1 < NRun; r += NT) uns |= m.k0[r] > m.k0[r + 1];
    if (__syncthreads_or(uns) && wg_sort<NT>(m.k0, m.v0, m.k1, m.v1, NRun, lds)) ov = m.v1;
  }
  for (uint32_t j = t; j < NRun; j += NT) {
    const uint32_t r = ov[j];
    m.Rord[j] = r;
    m.Rord2[j] = r;
    m.Rpos[r] = j;
  }
  __syncthreads();
  mark(14);
  auto key = [&](uint32_t r) -> uint64_t { return ((uint64_t)m.Rc[r] << 32) | m.Rs[r]; };
  // 4 tie groups: one lane per group re-sorts it by the predecessors' current ranks
  for (uint32_t round = 0;; round++) {
    uint32_t flags = 0; // 1 changed, 2 too big
    for (uint32_t j = t; j < NRun; j += NT) {
      const uint64_t kj = key(m.Rord[j]);
      if (j > 0 && key(m.Rord[j - 1]) == kj) continue;
      uint32_t g1 = j + 1;
      while (g1 < NRun && key(m.Rord[g1]) == kj) g1++;
      if (g1 - j == 1) continue;
      if (g1 - j > 256) {
        flags |= 2;
        continue;
      }
      for (uint32_t q = j; q < g1; q++) {
        const uint32_t x = m.Rord[q], px = m.Rp[x];
        uint32_t z = q;
        while (z > j) {
          const uint32_t y = m.Rord2[z - 1], py = m.Rp[y];
          const bool before = px != NONE ? (py == NONE || m.Rpos[px] > m.Rpos[py]) : (py == NONE && m.Ru[x] < m.Ru[y]);
          if (!before) break;
          m.Rord2[z] = y;
          z--;
        }
        m.Rord2[z] = x;
      }
      for (uint32_t q = j; q < g1; q++) flags |= m.Rord2[q] != m.Rord[q];
    }
    const uint32_t f = __syncthreads_or(flags & 1) | (__syncthreads_or(flags & 2) << 1);
    if (f & 2) return false;
    if (!(f & 1)) break;
    if (round >= 16) return false;
    for (uint32_t j = t; j < NRun; j += NT) {
      const uint32_t r = m.Rord2[j];
      m.Rord[j] = r;
      m.Rpos[r] = j;
    }
    __syncthreads();
  }
  mark(15);
  // 5 Item-vs-GC ties consumed while <= 20 decoders are live: last rank (+1) per update,
  //   V = the smallest v with #{u : lu[u] >= v} <= 20, tail = ranks >= V - 1
  uint32_t lo = 1;
  if (U <= BIG_LU_LDS && NRun + 1 <= BIG_LU_LDS) {
    // in LDS: lu per update, then a histogram of lu; #{lu >= v} <= 20 <=> #{lu < v} >= U - 20,
    // so V is the first v >= 1 where the histogram's prefix reaches U - 20
    uint32_t *llu = (uint32_t *)lds, *hist = llu + BIG_LU_LDS;
    for (uint32_t u = t; u < BIG_LU_LDS; u += NT) {
      llu[u] = 0;
      hist[u] = 0;
    }
    if (t == 0) sc[4] = NRun + 1;
    __syncthreads();
    for (uint32_t j = t; j < NRun; j += NT) atomicMax(&llu[m.Ru[m.Rord[j]]], j + 1);
    __syncthreads();
    for (uint32_t u = t; u < U; u += NT) atomicAdd(&hist[llu[u]], 1u);
    __syncthreads();
    constexpr uint32_t C = BIG_LU_LDS / NT; // histogram slots per lane, contiguous
    uint32_t csum = 0;
    for (uint32_t q = 0; q < C; q++) csum += hist[t * C + q];
    uint32_t T;
    uint32_t pre = bscan_sum<NT>(csum, ws, T);
    const uint32_t goal = U > 20 ? U - 20 : 0;
    for (uint32_t q = 0; q < C; q++) {
      const uint32_t v = t * C + q; // prefix(v) = pre = #{lu < v}
      if (v >= 1 && v <= NRun + 1 && pre >= goal) {
        atomicMin(&sc[4], v);
        break;
      }
      pre += hist[v];
    }
    __syncthreads();
    lo = sc[4];
    __syncthreads();
  } else {
    for (uint32_t u = t; u < U; u += NT) m.lu[u] = 0;
    __syncthreads();
    for (uint32_t j = t; j < NRun; j += NT) atomicMax(&m.lu[m.Ru[m.Rord[j]]], j + 1);
    __syncthreads();
    uint32_t hi = NRun + 1;
    while (lo < hi) { // uniform
      const uint32_t mid = (lo + hi) >> 1;
      uint32_t c = 0, T;
      for (uint32_t u = t; u < U; u += NT) c += m.lu[u] >= mid;
      bscan_sum<NT>(c, ws, T);
      if (T <= 20) hi = mid;
      else lo = mid + 1;
    }
  }
  const uint32_t V = lo;
  for (uint32_t j = t; j < NRun; j += NT) {
    const uint32_t r = m.Rord[j];
    const uint64_t kj = key(r);
    if (j > 0 && key(m.Rord[j - 1]) == kj) continue;
    uint32_t g1 = j + 1, kinds = 1u << m.Rk[r];
    while (g1 < NRun && key(m.Rord[g1]) == kj) kinds |= 1u << m.Rk[m.Rord[g1++]];
    if ((kinds & 3) == 3 && g1 >= V) bad = 1; // last rank g1 - 1 >= V - 1
  }
  if (__syncthreads_or(bad)) return false;
  // 6 sorted block positions: runs in rank order, blocks in run order
  uint32_t acc = 0;
  for (uint32_t base = 0; base < NRun; base += NT) {
    const uint32_t j = base + t;
    const uint32_t n = j < NRun ? m.Rn[m.Rord[j]] : 0;
    uint32_t T;
    const uint32_t pre = bscan_sum<NT>(n, ws, T);
    if (j < NRun) m.Roff[j] = acc + pre;
    acc += T;
  }
  __syncthreads();
  for (uint32_t j = t; j < NB; j += NT) {
    const uint32_t r = m.rr[j];
    m.sord[m.Roff[m.Rpos[r]] + (j - m.Rb[r])] = j;
  }
  __syncthreads();
  (void)sc;
  return true;
}

// ------------------------------------------------------------------ DeleteSet union by bitmap
// IdSet::merge then squash (yrs/src/id_set.rs:129-164, 385-395) leaves, per client, the
// maximal unions of overlapping or adjacent ranges: exactly the maximal runs of set bits once
// every range is set in a bitmap over the client's clock window (k_lean's DeleteSet,
// ymerge_lean.hip phase 4).  For the few-client documents whose windows fit LDS (C4: 1-4
// clients, windows of a few thousand clocks) this replaces the key pass, the range sort over
// HBM tables and the two union passes: one pass sets the windows, one sets the bits, one
// finds the runs, one sizes them and one writes them.
// d_client: the D (<= 64) distinct live clients ascending; d_ord: ranks in yrs' table order.
// pc: >= 9 * 64 LDS words; bm: BIG_BM_WORDS LDS words; cl: BIG_BM_COMP component pairs in
// LDS; chead / cend: the same in HBM when there are more components.
// Returns 0: not this shape (the sort path runs); DSB_ROOM: the DeleteSet does not fit the
// slot's `room` bytes (exact engine); else 1 + the DeleteSet's bytes, written at dso.
constexpr uint32_t BIG_BM_WORDS = 6144, BIG_BM_COMP = 2048, DSB_ROOM = 0xFFFFFFFFu;
template <int NT>
__device__ __noinline__ uint32_t big_ds_bitmap(const uint32_t *ri, const uint32_t *rs, const uint32_t *re,
                                               const uint32_t *et, const uint32_t *ec, uint32_t NR, uint32_t D,
                                               const uint32_t *d_client, const uint32_t *d_ord, uint32_t *pc,
                                               uint32_t *bm, uint32_t *cl, uint32_t *chead, uint32_t *cend,
                                               uint32_t *ws, uint8_t *dso, uint64_t room) {
  const uint32_t t = threadIdx.x;
  uint32_t *lo = pc, *hi = pc + 64, *woff = pc + 128, *nw = pc + 192, *ncomp = pc + 256, *cbase = pc + 320,
           *bytes = pc + 384, *bpre = pc + 448, *eoff = pc + 512, *misc = pc + 576;
  auto rank_of = [&](uint32_t c) -> uint32_t {
    uint32_t a = 0, z = D;
    while (a < z) {
      const uint32_t mid = (a + z) >> 1;
      if (d_client[mid] < c) a = mid + 1;
      else z = mid;
    }
    return a;
  };
  if (t < 64) {
    lo[t] = 0xFFFFFFFFu;
    hi[t] = 0;
    ncomp[t] = 0;
    bytes[t] = 0;
  }
  __syncthreads();
  // 1 windows: [min start, max end) of every client's live ranges; an empty range -> sort path
  uint32_t bad = 0;
  for (uint32_t j = t; j < NR; j += NT) {
    const uint32_t x = ri[j];
    if (!(et[x] & 0x80000000u)) continue;
    const uint32_t s = rs[j], e = re[j];
    if (e <= s) {
      bad = 1;
      continue;
    }
    const uint32_t r = rank_of(ec[x]);
    atomicMin(&lo[r], s);
    atomicMax(&hi[r], e);
  }
  if (__syncthreads_or(bad)) return 0;
  if (t == 0) { // word offsets, a zero word after every window (runs never cross clients)
    uint32_t acc = 0;
    for (uint32_t r = 0; r < D; r++) {
      const uint32_t n = lo[r] < hi[r] ? ((hi[r] - 1) >> 5) - (lo[r] >> 5) + 1 : 0;
      lo[r] &= ~31u;
      woff[r] = acc;
      nw[r] = n;
      acc += n + 1;
    }
    misc[0] = acc;
  }
  __syncthreads();
  const uint32_t W = misc[0];
  if (W > BIG_BM_WORDS) return 0;
  for (uint32_t q = t; q < W; q += NT) bm[q] = 0;
  __syncthreads();
  // 2 every live range into its client's window
  for (uint32_t j = t; j < NR; j += NT) {
    const uint32_t x = ri[j];
    if (!(et[x] & 0x80000000u)) continue;
    const uint32_t r = rank_of(ec[x]), wo = woff[r];
    uint32_t a = rs[j] - lo[r];
    const uint32_t z = re[j] - lo[r];
    while (a < z) {
      const uint32_t wi = a >> 5, bo = a & 31, nb = (z - a < 32 - bo) ? z - a : 32 - bo;
      atomicOr(&bm[wo + wi], (nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1)) << bo);
      a += nb;
    }
  }
  __syncthreads();
  // word -> client rank (the window holding word q; gap words have no bits)
  auto word_rank = [&](uint32_t q) -> uint32_t {
    uint32_t a = 0, z = D;
    while (a + 1 < z) {
      const uint32_t mid = (a + z) >> 1;
      if (woff[mid] <= q) a = mid;
      else z = mid;
    }
    return a;
  };
  // 3 runs: count per client, then starts / ends at their global component index
  for (uint32_t q = t; q < W; q += NT) {
    const uint32_t bits = bm[q], prev = q ? bm[q - 1] >> 31 : 0;
    const uint32_t stb = bits & ~((bits << 1) | prev);
    if (stb) atomicAdd(&ncomp[word_rank(q)], (uint32_t)__builtin_popcount(stb));
  }
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    for (uint32_t r = 0; r < D; r++) {
      cbase[r] = acc;
      acc += ncomp[r];
    }
    misc[1] = acc;
  }
  __syncthreads();
  const uint32_t NCOMP = misc[1];
  uint32_t *cs = NCOMP <= BIG_BM_COMP ? cl : chead, *ce = NCOMP <= BIG_BM_COMP ? cl + BIG_BM_COMP : cend;
  {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < W; base += NT) {
      const uint32_t q = base + t;
      const bool v = q < W;
      const uint32_t bits = v ? bm[q] : 0, prev = v && q ? bm[q - 1] >> 31 : 0;
      const uint32_t nxt = v && q + 1 < W ? bm[q + 1] & 1 : 0;
      const uint32_t stb = bits & ~((bits << 1) | prev), enb = bits & ~((bits >> 1) | (nxt << 31));
      uint32_t T;
      const uint32_t cb = carry + bscan_sum<NT>((uint32_t)__builtin_popcount(stb), ws, T);
      carry += T;
      if (bits) {
        const uint32_t r = word_rank(q), clk0 = lo[r] + 32 * (q - woff[r]);
        uint32_t x = stb;
        while (x) {
          const uint32_t bp = (uint32_t)__builtin_ctz(x);
          cs[cb + (uint32_t)__builtin_popcount(stb & ((1u << bp) - 1))] = clk0 + bp;
          x &= x - 1;
        }
        x = enb;
        while (x) {
          const uint32_t bp = (uint32_t)__builtin_ctz(x);
          const uint32_t upto = bp == 31 ? stb : (stb & ((2u << bp) - 1));
          ce[cb + (uint32_t)__builtin_popcount(upto) - 1] = clk0 + bp + 1;
          x &= x - 1;
        }
      }
    }
  }
  __syncthreads();
  auto comp_rank = [&](uint32_t k) -> uint32_t { // the client of component k (last r with cbase <= k, ncomp > 0)
    uint32_t a = 0, z = D;
    while (a + 1 < z) {
      const uint32_t mid = (a + z) >> 1;
      if (cbase[mid] <= k) a = mid;
      else z = mid;
    }
    while (a + 1 < D && cbase[a + 1] <= k) a++; // (ties: clients without components)
    return a;
  };
  // 4 bytes per client, entry offsets in yrs' table order (IdSet encode, id_set.rs:398-410)
  for (uint32_t k = t; k < NCOMP; k += NT) {
    const uint32_t a = cs[k];
    atomicAdd(&bytes[comp_rank(k)], (uint32_t)(varlen(a) + varlen(ce[k] - a)));
  }
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    for (uint32_t r = 0; r < D; r++) {
      bpre[r] = acc;
      acc += bytes[r];
    }
    uint32_t pos = varlen(D);
    for (uint32_t i = 0; i < D; i++) {
      const uint32_t r = d_ord[i];
      eoff[r] = pos;
      pos += varlen(d_client[r]) + varlen(ncomp[r]) + bytes[r];
    }
    misc[2] = pos;
  }
  __syncthreads();
  const uint32_t dsz = misc[2];
  if (dsz > room) return DSB_ROOM;
  // 5 write: D, per client (client, ranges), the components at their offsets
  if (t == 0) {
    Writer w{dso, 0};
    w_var(w, D);
  }
  if (t < D) {
    Writer w{dso, eoff[t]};
    w_var(w, d_client[t]);
    w_var(w, ncomp[t]);
  }
  uint32_t carry = 0;
  for (uint32_t base = 0; base < NCOMP; base += NT) {
    const uint32_t k = base + t;
    const bool v = k < NCOMP;
    const uint32_t a = v ? cs[k] : 0, ln = v ? ce[k] - a : 0;
    const uint32_t sz = v ? varlen(a) + varlen(ln) : 0;
    uint32_t T;
    const uint32_t P = carry + bscan_sum<NT>(sz, ws, T);
    carry += T;
    if (v) {
      const uint32_t r = comp_rank(k);
      Writer w{dso, eoff[r] + varlen(d_client[r]) + varlen(ncomp[r]) + (P - bpre[r])};
      w_var(w, a);
      w_var(w, ln);
    }
  }
  return 1 + dsz;
}

// ------------------------------------------------------------------ k_big_merge
template <int NT> struct BigShared {
  uint32_t ws[2 * (NT / 64) + 8];
  uint64_t ws64[NT / 64 + 2];
  uint32_t sc[32];
  unsigned long long err;
  __align__(16) uint8_t un[BIG_UNION + 64];
};

constexpr uint32_t BIG_COPY_MIN = 1024, BIG_COPY_N = 32;
template <int NT, int OCC>
__global__ void __launch_bounds__(NT, OCC) k_big_merge(BatchIn b, const uint32_t *counts, const uint64_t *scr_off,
                                                       uint32_t *scratch, FastOut o, uint32_t flags) {
  const bool big_ds_bm = !(flags & 1); // DeleteSet union by bitmap when it fits (env YMERGE_BIG_DSBM=0: off)
  ym_set_grammar(b.v1x);
  const uint32_t d = o.big_list[blockIdx.x];
  if (d >= b.n_docs || o.path[d] != 2) return;
  __shared__ BigShared<NT> S;
  // verbatim blocks of >= BIG_COPY_MIN bytes of a write tile: copied by the whole workgroup
  // after the tile (one lane copying a 69 KB pasted string held a trace document ~4 M cycles)
  __shared__ uint32_t s_nbig, s_bl[BIG_COPY_N];
  __shared__ uint64_t s_bd[BIG_COPY_N], s_bs[BIG_COPY_N];
  const uint32_t t = threadIdx.x;
  uint32_t *ws = S.ws, *sc = S.sc;
  const uint32_t NB = counts[4 * d + 1], NE = counts[4 * d + 2], NR = counts[4 * d + 3];
  const uint64_t u0 = b.doc_upd[d], u1 = b.doc_upd[d + 1];
  const uint32_t U = (uint32_t)(u1 - u0);
  BigMem m = big_carve(scratch + scr_off[d], NB, NE, NR, U);
  big_uniform(m);
  const uint64_t B0 = b.upd_off[u0];
  const uint32_t nbytes = (uint32_t)(b.upd_off[u1] - B0);
  const uint8_t *in = b.bytes + B0;
  const uint64_t slot = 2 * B0 + 64ull * d;
  const uint64_t cap = 2ull * nbytes + 64;
  uint8_t *out = o.out + slot;
  bool om = false; // overlap mode: m.sord holds the run order of big_run_order
  // diagnostic runs only (YMERGE_STAMPS=1 sets o.stamps): s_memtime per phase, slot 7 = marker
  auto stamp = [&](uint32_t k) {
    if (o.stamps) {
      __syncthreads();
      if (t == 0) {
        o.stamps[(size_t)d * 16 + k] = __builtin_amdgcn_s_memtime();
        o.stamps[(size_t)d * 16 + 7] = 0xB16;
      }
    }
  };
  stamp(0);
  // sub-phase marks (slots 8..12): classify pass 0 / run order, DeleteSet table / range sort / union
  auto mark = [&](uint32_t k) {
    if (o.stamps) {
      __syncthreads();
      if (t == 0) o.stamps[(size_t)d * 16 + k] = __builtin_amdgcn_s_memtime();
    }
  };
  auto finish = [&](uint8_t p, uint8_t st, uint64_t len) {
    if (t == 0) {
      if (p == 1) {
        atomicAdd(&o.npath[1], 1u);
        atomicAdd(&o.npath[4], 1u); // tiled -> exact engine
      } else if (om) {
        atomicAdd(&o.npath[3], 1u); // written in overlap mode
      }
      o.path[d] = p;
      o.status[d] = st;
      o.out_len[d] = len;
      o.out_start[d] = slot;
    }
  };

  // ---- 1 gather: rounds of NT updates; the round's counts are scanned and every lane
  //      writes its records at the scanned positions (records of k_decode, overflow words,
  //      or a walk of the update for the shapes k_decode left to a later pass)
  {
    uint32_t NBr = 0, NEr = 0, NRr = 0;
    if (t == 0) sc[5] = 0;
    __syncthreads();
    uint64_t g_rec = 0, g_scan = 0, g_write = 0, g_slow = 0; // diagnostic sub-phase sums (thread 0, stamps only)
    uint64_t g_r0 = 0, g_w0 = 0, g_rmax = 0, g_wmax = 0;      // round 0 / slowest later round
    for (uint32_t r0 = 0; r0 < U; r0 += NT) {
      const uint64_t tg0 = o.stamps ? __builtin_amdgcn_s_memtime() : 0;
      const uint32_t i = r0 + t;
      uint32_t ubase = 0, ulen = 0, shape = 0, w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0, w5 = 0;
      uint32_t snb = 0, sne = 0, snr = 0;
      bool walk = false;
      if (i < U) {
        const uint64_t a0 = b.upd_off[u0 + i], a1 = b.upd_off[u0 + i + 1];
        ubase = (uint32_t)(a0 - B0);
        ulen = (uint32_t)(a1 - a0);
        const uint2 *rp = (const uint2 *)(b.rec + (size_t)(u0 + i) * REC_WORDS);
        const uint2 x0 = rp[0], x1 = rp[1], x2 = rp[2];
        w0 = x0.x;
        w1 = x0.y;
        w2 = x1.x;
        w3 = x1.y;
        w4 = x2.x;
        w5 = x2.y;
        if (w0 & REC_SLOW) {
          uint32_t w[6];
          walk_record_hbm(in + ubase, ulen, w);
          w0 = w[0];
          w1 = w[1];
          w2 = w[2];
          w3 = w[3];
          w4 = w[4];
          w5 = w[5];
        }
        shape = (w0 >> 10) & 3;
        if (shape == REC_BLOCK) snb = 1;
        else if (shape == REC_DS) {
          sne = 1;
          snr = (w0 >> 12) & 3;
        } else if (shape == REC_COMPLEX) {
          snb = w1;
          sne = w2;
          snr = w3;
          walk = !(w0 & REC_OVF);
        }
      }
      if (o.stamps) {
        __syncthreads();
      }
      const uint64_t tg1 = o.stamps ? __builtin_amdgcn_s_memtime() : 0;
      uint64_t T0, T1;
      const uint64_t p0 = bscan_sum64<NT>((uint64_t)snb | ((uint64_t)sne << 32), S.ws64, T0);
      const uint64_t p1 = bscan_sum64<NT>((uint64_t)snr, S.ws64, T1);
      const uint32_t pb = NBr + (uint32_t)p0, pe = NEr + (uint32_t)(p0 >> 32), pr = NRr + (uint32_t)p1;
      NBr += (uint32_t)T0;
      NEr += (uint32_t)(T0 >> 32);
      NRr += (uint32_t)T1;
      const uint64_t tg2 = o.stamps ? __builtin_amdgcn_s_memtime() : 0;
      if (o.stamps) {
        g_rec += tg1 - tg0;
        g_scan += tg2 - tg1;
        if (r0 == 0) g_r0 = tg1 - tg0;
        else g_rmax = g_rmax > tg1 - tg0 ? g_rmax : tg1 - tg0;
      }
      uint32_t co = 0; // 1: this lane's record list is copied by the workgroup
      if (i < U) {
      if (shape == REC_BLOCK) {
        m.bc[pb] = w1;
        m.bk[pb] = w2;
        m.bl[pb] = w3;
        m.bp[pb] = ubase + w4;
        m.bm[pb] = w5;
        m.bu[pb] = i;
      } else if (shape == REC_DS) {
        m.ec[pe] = w1;
        m.et[pe] = 0x80000000u | (i << 8);
        if (snr > 0) {
          m.rs[pr] = w2;
          m.re[pr] = w3;
          m.ri[pr] = pe;
        }
        if (snr > 1) {
          m.rs[pr + 1] = w4;
          m.re[pr + 1] = w5;
          m.ri[pr + 1] = pe;
        }
      } else if (shape == REC_COMPLEX && !walk && snb + sne + snr > BIG_COOP && (co = atomicAdd(&sc[5], 1u)) < 8) {
        // a long record list (k_decode_huge: thousands of blocks in one update) is copied by
        // the whole workgroup after this round's writes instead of by this lane
        uint32_t *ce = (uint32_t *)S.un + 8 * co;
        ce[0] = i;
        ce[1] = pb;
        ce[2] = pe;
        ce[3] = pr;
        ce[4] = w4;
        ce[5] = snb;
        ce[6] = sne;
        ce[7] = snr;
        co = 1;
      } else if (shape == REC_COMPLEX && !walk) {
        co = 0;
        const uint32_t *ov = b.ovf + w4;
        for (uint32_t k = 0; k < snb; k++) {
          m.bc[pb + k] = ov[5 * k];
          m.bk[pb + k] = ov[5 * k + 1];
          m.bl[pb + k] = ov[5 * k + 2];
          m.bp[pb + k] = ubase + ov[5 * k + 3];
          m.bm[pb + k] = ov[5 * k + 4];
          m.bu[pb + k] = i;
        }
        ov += 5 * snb;
        for (uint32_t k = 0; k < sne; k++) {
          m.ec[pe + k] = ov[k];
          m.et[pe + k] = ov[sne + k] | (i << 8); // table code from k_decode
        }
        ov += 2 * sne;
        for (uint32_t k = 0; k < snr; k++) {
          m.rs[pr + k] = ov[3 * k];
          m.re[pr + k] = ov[3 * k + 1];
          m.ri[pr + k] = pe + ov[3 * k + 2];
        }
      } else if (shape == REC_COMPLEX) {
        FastFill f{m.bc, m.bk, m.bl, m.bp, m.bm, m.ec, m.et, m.rs, m.re, m.ri, i, ubase, pb, pe, pr, 0};
        fill_hbm(in + ubase, ulen, &f);
        for (uint32_t k = 0; k < snb; k++) m.bu[pb + k] = i;
      }
      }
      if (__syncthreads_or(co == 1)) { // the deferred long record lists, one after another
        const uint32_t nco = sc[5] < 8 ? sc[5] : 8;
        for (uint32_t q = 0; q < nco; q++) {
          const uint32_t *ce = (const uint32_t *)S.un + 8 * q;
          const uint32_t ci = ce[0], cb = ce[1], cE = ce[2], cr = ce[3], nb2 = ce[5], ne2 = ce[6], nr2 = ce[7];
          const uint32_t cub = (uint32_t)(b.upd_off[u0 + ci] - B0);
          const uint32_t *ov = b.ovf + ce[4];
          for (uint32_t k = t; k < nb2; k += NT) {
            m.bc[cb + k] = ov[5 * k];
            m.bk[cb + k] = ov[5 * k + 1];
            m.bl[cb + k] = ov[5 * k + 2];
            m.bp[cb + k] = cub + ov[5 * k + 3];
            m.bm[cb + k] = ov[5 * k + 4];
            m.bu[cb + k] = ci;
          }
          const uint32_t *oe = ov + 5 * nb2;
          for (uint32_t k = t; k < ne2; k += NT) {
            m.ec[cE + k] = oe[k];
            m.et[cE + k] = oe[ne2 + k] | (ci << 8);
          }
          const uint32_t *orr = oe + 2 * ne2;
          for (uint32_t k = t; k < nr2; k += NT) {
            m.rs[cr + k] = orr[3 * k];
            m.re[cr + k] = orr[3 * k + 1];
            m.ri[cr + k] = cE + orr[3 * k + 2];
          }
        }
        __syncthreads();
        if (t == 0) sc[5] = 0;
        __syncthreads();
      }
      if (o.stamps) {
        __syncthreads();
        const uint64_t gw = __builtin_amdgcn_s_memtime() - tg2;
        g_write += gw;
        if (r0 == 0) g_w0 = gw;
        else g_wmax = g_wmax > gw ? g_wmax : gw;
      }
    }
    if (o.stamps && t == 0) {
      (void)g_rec;
      (void)g_scan;
      (void)g_write;
      (void)g_r0;
      (void)g_rmax;
      (void)g_w0;
      (void)g_wmax;
    }
  }
  __syncthreads();

  stamp(1);
  // ---- 2 sort blocks by (client desc, clock asc, input order)
  const uint32_t *sval = m.v0;
  bool ident = true;
  {
    uint32_t bad = 0;
    for (uint32_t j = t; j + 1 < NB; j += NT) {
      const uint64_t a = ((uint64_t)(~m.bc[j]) << 32) | m.bk[j], c = ((uint64_t)(~m.bc[j + 1]) << 32) | m.bk[j + 1];
      if (a > c) bad = 1;
    }
    ident = !__syncthreads_or(bad);
    // Few clients (the usual case: a handful of editors): stable counting sort by client
    // rank in tiles, then a clock-order check per client run; the general stable sort runs
    // only when that check fails or there are more than 8 clients.
    bool counted = false;
    if (!ident && NB < (1u << 25)) {
      uint64_t *btab = (uint64_t *)S.un; // [64] client << 32 | rank, ~0 = empty
      for (uint32_t i = t; i < 64; i += NT) btab[i] = ~0ull;
      if (t == 0) sc[3] = 0;
      __syncthreads();
      uint32_t ovf = 0;
      for (uint32_t j = t; j < NB && !ovf; j += NT) {
        const uint32_t c = m.bc[j];
        if (j > 0 && m.bc[j - 1] == c) continue;
        uint32_t h = mix32(c) >> 26;
        for (uint32_t probe = 0;; probe++) {
          if (probe == 64) {
            ovf = 1;
            break;
          }
          uint64_t cur = btab[h];
          if (cur == ~0ull) {
            const uint64_t prev = atomicCAS((unsigned long long *)&btab[h], ~0ull, (unsigned long long)c << 32);
            if (prev == ~0ull) {
              atomicAdd(&sc[3], 1u);
              break;
            }
            cur = prev;
          }
          if ((uint32_t)(cur >> 32) == c) break;
          h = (h + 1) & 63;
        }
      }
      ovf = __syncthreads_or(ovf);
      const uint32_t ncl = sc[3];
      if (!ovf && ncl <= 8) {
        // rank = number of distinct clients greater than this one (descending client order)
        const uint64_t mine = t < 64 ? btab[t] : ~0ull;
        uint32_t r = 0;
        if (mine != ~0ull)
          for (uint32_t q = 0; q < 64; q++) {
            const uint64_t o2 = btab[q];
            r += (o2 != ~0ull && (uint32_t)(o2 >> 32) > (uint32_t)(mine >> 32));
          }
        __syncthreads();
        if (mine != ~0ull) btab[t] = (mine & 0xFFFFFFFF00000000ull) | r;
        __syncthreads();
        auto rank_of = [&](uint32_t c) -> uint32_t {
          uint32_t h = mix32(c) >> 26;
          while ((uint32_t)(btab[h] >> 32) != c) h = (h + 1) & 63;
          return (uint32_t)btab[h];
        };
        // rank totals (per-lane 16-bit fields: < 2^25 / NT elements per lane), rank starts
        uint64_t c0 = 0, c1 = 0;
        for (uint32_t j = t; j < NB; j += NT) {
          const uint32_t rr = rank_of(m.bc[j]);
          if (rr < 4) c0 += 1ull << (16 * rr);
          else c1 += 1ull << (16 * (rr - 4));
        }
        uint32_t start[8], carry[8];
        {
          uint32_t *rtot = (uint32_t *)(S.un + 64 * 8); // [8] LDS rank totals
          if (t < 8) rtot[t] = 0;
          __syncthreads();
#pragma unroll
          for (uint32_t q = 0; q < 8; q++) {
            const uint32_t v = (uint32_t)(q < 4 ? (c0 >> (16 * q)) & 0xFFFF : (c1 >> (16 * (q - 4))) & 0xFFFF);
            if (v) atomicAdd(&rtot[q], v);
          }
          __syncthreads();
          uint32_t acc = 0;
#pragma unroll
          for (uint32_t q = 0; q < 8; q++) {
            start[q] = acc;
            carry[q] = 0;
            acc += rtot[q];
          }
        }
        // tiles in input order: within-tile prefix per rank (two packed scans), then place
        for (uint32_t base = 0; base < NB; base += NT) {
          const uint32_t j = base + t;
          const bool valid = j < NB;
          const uint32_t rr = valid ? rank_of(m.bc[j]) : 0;
          const uint64_t i0 = valid && rr < 4 ? 1ull << (16 * rr) : 0, i1 = valid && rr >= 4 ? 1ull << (16 * (rr - 4)) : 0;
          uint64_t T0, T1;
          const uint64_t p0 = bscan_sum64<NT>(i0, S.ws64, T0), p1 = bscan_sum64<NT>(i1, S.ws64, T1);
          if (valid) {
            const uint32_t within = rr < 4 ? (uint32_t)((p0 >> (16 * rr)) & 0xFFFF) : (uint32_t)((p1 >> (16 * (rr - 4))) & 0xFFFF);
            uint32_t st = 0, ca = 0;
#pragma unroll
            for (uint32_t q = 0; q < 8; q++)
              if (q == rr) {
                st = start[q];
                ca = carry[q];
              }
            const uint32_t pos = st + ca + within;
            m.v1[pos] = j;
            m.k1[pos] = ((uint64_t)(~m.bc[j]) << 32) | m.bk[j];
          }
#pragma unroll
          for (uint32_t q = 0; q < 8; q++)
            carry[q] += q < 4 ? (uint32_t)((T0 >> (16 * q)) & 0xFFFF) : (uint32_t)((T1 >> (16 * (q - 4))) & 0xFFFF);
        }
        __syncthreads();
        uint32_t bad2 = 0;
        for (uint32_t j = t; j + 1 < NB; j += NT)
          if (m.k1[j] > m.k1[j + 1]) bad2 = 1;
        counted = !__syncthreads_or(bad2);
        if (counted) sval = m.v1;
      }
    }
    if (!ident && !counted) {
      for (uint32_t j = t; j < NB; j += NT) {
        m.k0[j] = ((uint64_t)(~m.bc[j]) << 32) | m.bk[j];
        m.v0[j] = j;
      }
      __syncthreads();
      if (wg_sort<NT>(m.k0, m.v0, m.k1, m.v1, NB, S.un)) sval = m.v1;
    }
  }
  auto srt = [&](uint32_t j) -> uint32_t { return om ? m.sord[j] : (ident ? j : sval[j]); };

  stamp(2);
  // ---- 3 classify (tiles of NT sorted positions, carries between tiles):
  //      running end E (segmented max), keep / Skip / drop; first pass: a partial overlap
  //      or a same-clock block that is not a duplicate of the kept one -> overlap mode,
  //      which classifies again in run order and keeps the straddling block spliced at E
  //      (flag 4, offset E - clock); emitted blocks per client segment
  uint32_t NC = 0; // client segments
  for (int pass = 0; pass < 2; pass++) {
    uint32_t cE = 0, cK = 0, cS = 0, cH = 0; // carries: running end, last kept (j+1), emitted count, heads
    uint32_t viol = 0, pan = 0, zl = 0, bsp = 0;
    for (uint32_t base = 0; base < NB; base += NT) {
      const uint32_t j = base + t;
      const bool valid = j < NB;
      uint32_t r = 0, c = 0, k = 0, l = 0, mt = 0;
      bool hd = false;
      if (valid) {
        r = srt(j);
        c = m.bc[r];
        k = m.bk[r];
        l = m.bl[r];
        mt = m.bm[r];
        hd = j == 0 || m.bc[srt(j - 1)] != c;
      }
      const uint32_t e = k + l;
      uint32_t pf, pv;
      bscan_seg<NT, OpMax>(valid && hd, valid ? e : 0, ws, pf, pv);
      const uint32_t E = hd ? 0 : (pf ? pv : (cE > pv ? cE : pv));
      uint32_t flag = 0;
      if (valid) {
        if (l == 0) zl = 1; // zero-length GC: exact engine
        if (hd || k >= E) {
          flag = 1;
          if (!hd && k > E) flag |= 2;
        } else if (e > E) {
          if (!om) {
            viol = 1; // partial overlap
          } else {
            flag = 1 | 4;
            m.fO[j] = E - k;
            if (!big_splice_ok(in, nbytes, m.bp[r], l, E - k)) bsp = 1;
          }
        }
      }
      // last kept position (j + 1) before j within the segment
      uint32_t qf, qv;
      bscan_seg<NT, OpMax>(valid && hd, (flag & 1) ? j + 1 : 0, ws, qf, qv);
      const uint32_t last = hd ? 0 : (qf ? qv : (cK > qv ? cK : qv));
      if (!om && valid && !(flag & 1) && last) {
        const uint32_t kr = srt(last - 1);
        if (m.bk[kr] == k) { // same start: must be an exact duplicate (kind, length, bytes)
          const uint32_t la = m.bm[kr] >> 8, lb = mt >> 8;
          bool same = la == lb && (m.bm[kr] & 3) == (mt & 3) && m.bl[kr] == l;
          if (same) same = equal_window(in + m.bp[kr], in + m.bp[r], la);
          if (!same) viol = 1;
        }
      }
      if (valid && (flag & 5) == 1 && (mt & 8)) pan = 1; // yrs panics encoding a kept String off a char boundary
      // emitted blocks per client segment (kept + Skips) and the segment rank
      const uint32_t cnt = (flag & 1) + ((flag >> 1) & 1);
      uint32_t sf, sv2;
      bscan_seg<NT, OpSum>(valid && hd, cnt, ws, sf, sv2);
      const uint32_t run_before = hd ? 0 : (sf ? sv2 : cS + sv2);
      uint32_t HT;
      const uint32_t hpre = bscan_sum<NT>(valid && hd ? 1u : 0u, ws, HT);
      const uint32_t rank = cH + hpre + (hd ? 1 : 0); // 1-based rank of j's segment
      if (valid) {
        m.fE[j] = E;
        m.fF[j] = flag;
        const bool tail = j + 1 == NB || m.bc[srt(j + 1)] != c;
        if (tail) m.sseg[rank - 1] = run_before + cnt;
      }
      // carries for the next tile: values after the last element of this tile
      const uint32_t lastj = (NB - base < (uint32_t)NT ? NB - base : (uint32_t)NT) - 1;
      if (t == lastj) {
        sc[0] = hd ? e : (E > e ? E : e);
        sc[1] = (flag & 1) ? j + 1 : last;
        sc[2] = run_before + cnt;
      }
      __syncthreads();
      cE = sc[0];
      cK = sc[1];
      cS = sc[2];
      cH += HT;
      // pass 0 stops at the first tile with a partial overlap: overlap mode classifies every
      // block again (pass 1), so the rest of this pass would be discarded
      if (!om && __syncthreads_or(viol)) break;
      __syncthreads();
    }
    NC = cH;
    // (__syncthreads_or returns 0/1: one barrier per flag)
    const uint32_t vp = (__syncthreads_or(viol) ? 1u : 0u) | (__syncthreads_or(pan) ? 2u : 0u) |
                        (__syncthreads_or(zl | bsp) ? 4u : 0u);
    if (vp & 4) { // zero-length GC, splice the device does not restate: exact engine
      finish(1, 0, 0);
      return;
    }
    if (vp & 1) { // partial overlap / same-clock mismatch: the run order of the yrs loop
      mark(8);
      // (a copy: the callee takes the tables by reference, which would otherwise keep the
      // kernel's own BigMem in scratch memory for every access of every phase)
      BigMem mc = m;
      const bool ro = big_run_order<NT>(b, u0, U, B0, NB, mc, ws, sc, S.un, o.stamps ? o.stamps + (size_t)d * 16 : nullptr);
      mark(9);
      if (!ro) {
        finish(1, 0, 0);
        return;
      }
      om = true;
      continue;
    }
    if (vp & 2) {
      finish(0, E_PANIC, 0);
      return;
    }
    break;
  }

  stamp(3);
  // ---- 4 sizes, offsets, write (LDS-staged per tile when the tile's bytes fit)
  uint64_t blocks_size = varlen(NC);
  bool ovf = false;
  {
    if (t == 0 && blocks_size <= cap) {
      Writer w{out, 0};
      w_var(w, NC);
    }
    uint32_t cH = 0;
    for (uint32_t base = 0; base < NB; base += NT) {
      const uint32_t j = base + t;
      const bool valid = j < NB;
      uint32_t r = 0, c = 0, k = 0, l = 0, mt = 0, p = 0, E = 0, flag = 0, s = 0, cnt = 0;
      bool hd = false;
      if (valid) {
        r = srt(j);
        c = m.bc[r];
        k = m.bk[r];
        l = m.bl[r];
        mt = m.bm[r];
        p = m.bp[r];
        E = m.fE[j];
        flag = m.fF[j];
        hd = j == 0 || m.bc[srt(j - 1)] != c;
      }
      uint32_t HT;
      const uint32_t hpre = bscan_sum<NT>(valid && hd ? 1u : 0u, ws, HT);
      if (valid) {
        if (hd) {
          cnt = m.sseg[cH + hpre];
          s += varlen(cnt) + varlen(c) + varlen(k);
        }
        if (flag & 2) s += 1 + varlen(k - E);
        if (flag & 4) {
          Counter cn;
          emit_block(in, nbytes, p, c, k, l, m.fO[j], cn);
          s += (uint32_t)cn.n;
        } else if (flag & 1) {
          s += canon_size(in, nbytes, p, c, k, l, mt);
        }
      }
      cH += HT;
      uint64_t TT;
      const uint64_t pre = bscan_sum64<NT>((uint64_t)s, S.ws64, TT);
      const uint64_t o0 = blocks_size; // offset of this tile's first byte
      blocks_size += TT;
      if (blocks_size > cap) {
        ovf = true;
        break; // uniform
      }
      // stage the tile's bytes in LDS at the destination's 16-byte phase when they fit
      const uint32_t phase = (uint32_t)((uintptr_t)(out + o0) & 15);
      const bool staged = phase + TT <= BIG_UNION;
      uint8_t *dst = staged ? S.un + phase : out + o0;
      if (t == 0) s_nbig = 0;
      __syncthreads();
      if (valid && s) {
        Writer w{dst, pre};
        if (hd) {
          w_var(w, cnt);
          w_var(w, c);
          w_var(w, k);
        }
        if (flag & 2) {
          w.u8(10);
          w_var(w, k - E);
        }
        if (flag & 1) {
          if (flag & 4) {
            Writer w2 = w;
            emit_block(in, nbytes, p, c, k, l, m.fO[j], w2);
          } else if ((mt & 4) && !(mt & 8)) {
            Writer w2 = w;
            emit_block(in, nbytes, p, c, k, l, 0, w2);
          } else {
            const uint32_t bl = mt >> 8;
            uint32_t q = BIG_COPY_N;
            if (bl >= BIG_COPY_MIN) q = atomicAdd(&s_nbig, 1u);
            if (q < BIG_COPY_N) {
              s_bd[q] = (uint64_t)(w.p + w.n);
              s_bs[q] = (uint64_t)(in + p);
              s_bl[q] = bl;
            } else {
              copy_bytes16(w.p + w.n, in + p, bl);
            }
          }
        }
      }
      __syncthreads();
      {
        const uint32_t nbig = s_nbig < BIG_COPY_N ? s_nbig : BIG_COPY_N;
        for (uint32_t e = 0; e < nbig; e++) // 16-byte stores (ycopy.h)
          copy_coop((uint8_t *)s_bd[e], (const uint8_t *)s_bs[e], s_bl[e], t, NT);
      }
      if (staged) {
        __syncthreads();
        uint8_t *gbase = out + o0 - phase;
        const uint32_t span = phase + (uint32_t)TT, nch = (span + 15) >> 4;
        for (uint32_t q = t; q < nch; q += NT) {
          const uint32_t b0 = q << 4, lo = b0 < phase ? phase : b0, hi = b0 + 16 < span ? b0 + 16 : span;
          if (lo == b0 && hi == b0 + 16) *(uint4 *)(gbase + b0) = *(const uint4 *)(S.un + b0);
          else
            for (uint32_t z = lo; z < hi; z++) gbase[z] = S.un[z];
        }
      }
      __syncthreads();
    }
  }
  if (ovf) { // output larger than the slot: the exact engine writes it to the spill region
    finish(1, 0, 0);
    return;
  }

  stamp(4);
  // ---- 5 DeleteSet: distinct clients and first occurrence (LDS hash, 64-bit CAS insert,
  //      atomicMin on a hit), sorted by client; yrs' table order (IdSet::merge inserts in
  //      first-occurrence order, hashbrown layout); live ranges sorted by (client, start);
  //      segmented union; write
  uint64_t *dtab = (uint64_t *)S.un;                              // [BIG_DTAB]
  uint32_t *d_client = (uint32_t *)(S.un + BIG_OFF_DARR);         // 7 x [BIG_DCAP]
  uint32_t *d_first = d_client + BIG_DCAP, *d_ord = d_first + BIG_DCAP, *d_beg = d_ord + BIG_DCAP;
  uint32_t *r_ncomp = d_beg + BIG_DCAP, *r_off = r_ncomp + BIG_DCAP, *r_end = r_off + BIG_DCAP;
  uint8_t *lscr = S.un + BIG_OFF_SCR; // sort chunk / bitonic values / table slots
  for (uint32_t j = t; j < BIG_DTAB; j += NT) dtab[j] = ~0ull;
  __syncthreads();
  uint32_t tovf = 0;
  for (uint32_t j = t; j < NE && !tovf; j += NT) {
    const uint32_t et = m.et[j];
    if (!(et & 0x80000000u)) continue;
    const uint32_t c = m.ec[j];
    const uint64_t v = ((uint64_t)c << 32) | (et & 0x7FFFFFFFu);
    const uint32_t h0 = mix32(c) & (BIG_DTAB - 1);
    uint32_t h = h0;
    for (;;) {
      uint64_t cur = dtab[h];
      if (cur == ~0ull) {
        cur = atomicCAS((unsigned long long *)&dtab[h], ~0ull, (unsigned long long)v);
        if (cur == ~0ull) break;
      }
      if ((uint32_t)(cur >> 32) == c) {
        atomicMin((unsigned long long *)&dtab[h], (unsigned long long)v);
        break;
      }
      h = (h + 1) & (BIG_DTAB - 1);
      if (h == h0) {
        tovf = 1;
        break;
      }
    }
  }
  if (__syncthreads_or(tovf)) {
    finish(1, 0, 0);
    return;
  }
  // D distinct clients.  Few (the usual case): the occupied slots are compacted and one
  // wave sorts them in registers (by client, then the ranks by first occurrence); else the
  // whole table is bitonic-sorted twice (occupied slots first).
  uint32_t D;
  {
    uint32_t c = 0;
    for (uint32_t j = t; j < BIG_DTAB; j += NT) c += dtab[j] != ~0ull;
    uint32_t pre = bscan_sum<NT>(c, ws, D);
    if (D <= 64) {
      uint64_t *cmp = (uint64_t *)lscr;
      for (uint32_t j = t; j < BIG_DTAB; j += NT)
        if (dtab[j] != ~0ull) cmp[pre++] = dtab[j];
      __syncthreads();
      if (t < 64) {
        const uint64_t x = wave_bitonic64(t < D ? cmp[t] : ~0ull, t); // (client, first occurrence)
        if (t < D) {
          d_client[t] = (uint32_t)(x >> 32);
          d_first[t] = (uint32_t)x;
        }
        const uint64_t y = wave_bitonic64(t < D ? ((x & 0xFFFFFFFFull) << 32) | t : ~0ull, t);
        if (t < D) dtab[t] = y; // rank of the t-th first occurrence in the low half
      }
      __syncthreads();
    }
  }
  if (D > BIG_DCAP) {
    finish(1, 0, 0);
    return;
  }
  if (D > 64) {
    {
      uint32_t *tv = (uint32_t *)lscr; // values (unused by the order)
      for (uint32_t j = t; j < BIG_DTAB; j += NT) tv[j] = j;
      __syncthreads();
      bitonic_reg<NT>(dtab, tv, BIG_DTAB);
    }
    for (uint32_t j = t; j < D; j += NT) {
      d_client[j] = (uint32_t)(dtab[j] >> 32);
      d_first[j] = (uint32_t)dtab[j];
    }
    __syncthreads();
    // first-occurrence order of the ranks (dtab reused as keys: first << 32 | rank)
    for (uint32_t j = t; j < BIG_DTAB; j += NT) dtab[j] = j < D ? ((uint64_t)d_first[j] << 32) | j : ~0ull;
    {
      uint32_t *tv = (uint32_t *)lscr;
      for (uint32_t j = t; j < BIG_DTAB; j += NT) tv[j] = j;
      __syncthreads();
      bitonic_reg<NT>(dtab, tv, BIG_DTAB);
    }
  }
  // hashbrown emulation (single lane; D <= BIG_DCAP): slots hold rank + 1
  if (t == 0) {
    uint32_t *slot_arr = (uint32_t *)lscr; // 2 * BIG_DTAB u32
    uint32_t *tmp = slot_arr + BIG_DTAB;
    uint32_t buckets = 0, items = 0, growth = 0;
    auto ctrl_empty = [&](uint32_t idx) -> bool {
      if (idx < buckets) return slot_arr[idx] == 0;
      if (buckets < 16) return idx < 16 ? true : slot_arr[idx - 16] == 0;
      return slot_arr[idx - buckets] == 0;
    };
    auto find_slot = [&](uint32_t key) -> uint32_t {
      uint32_t mask = buckets - 1, pos = key & mask, stride = 0;
      for (;;) {
        for (uint32_t j = 0; j < 16; j++) {
          if (ctrl_empty(pos + j)) {
            const uint32_t index = (pos + j) & mask;
            if (slot_arr[index] != 0)
              for (uint32_t k = 0; k < buckets; k++)
                if (slot_arr[k] == 0) return k;
            return index;
          }
        }
        stride += 16;
        pos = (pos + stride) & mask;
      }
    };
    for (uint32_t i = 0; i < D; i++) {
      if (growth == 0) {
        const uint64_t full = buckets ? mask_to_cap(buckets - 1) : 0;
        const uint64_t need = items + 1;
        const uint32_t nb = (uint32_t)cap_to_buckets(need > full + 1 ? need : full + 1);
        for (uint32_t q = 0; q < buckets; q++) tmp[q] = slot_arr[q];
        const uint32_t ob = buckets;
        buckets = nb;
        for (uint32_t q = 0; q < buckets; q++) slot_arr[q] = 0;
        for (uint32_t q = 0; q < ob; q++)
          if (tmp[q]) slot_arr[find_slot(d_client[tmp[q] - 1])] = tmp[q];
        growth = (uint32_t)mask_to_cap(buckets - 1) - items;
      }
      const uint32_t rk = (uint32_t)dtab[i]; // rank of the i-th first occurrence
      slot_arr[find_slot(d_client[rk])] = rk + 1;
      items++;
      growth--;
    }
    uint32_t k = 0;
    for (uint32_t q = 0; q < buckets; q++)
      if (slot_arr[q]) d_ord[k++] = slot_arr[q] - 1;
  }
  __syncthreads();
  mark(10);
  if (D >= 1 && D <= 64 && big_ds_bm) {
    const uint32_t rb = big_ds_bitmap<NT>(m.ri, m.rs, m.re, m.et, m.ec, NR, D, d_client, d_ord, d_first,
                                          (uint32_t *)lscr, (uint32_t *)dtab, m.chead, m.cend, ws, out + blocks_size,
                                          cap - blocks_size);
    if (rb == DSB_ROOM) {
      finish(1, 0, 0);
      return;
    }
    if (rb) {
      stamp(5);
      finish(0, 0, blocks_size + (rb - 1));
      return;
    }
  }
  // live ranges sorted by (client, start, index).  One pass builds the keys, counts the
  // live ones and checks the order; four ranges per lane per trip with every load of the
  // trip issued before the first use (the loop was a chain of dependent HBM round trips)
  const uint64_t *dkey = m.k0;
  const uint32_t *dval = m.v0;
  uint32_t NL;
  {
    const uint32_t *__restrict__ g_ri = m.ri, *__restrict__ g_rs = m.rs, *__restrict__ g_et = m.et,
                   *__restrict__ g_ec = m.ec;
    uint64_t *__restrict__ g_k0 = m.k0;
    uint32_t *__restrict__ g_v0 = m.v0;
    const uint32_t lane = t & 63;
    uint32_t bad = 0, live_n = 0;
    constexpr uint32_t RB = 4;
    // few clients (D <= 64, ranks in LDS ascending by client): keys packed as (client rank,
    // start, index) in 6 + 32 + 26 bits -- distinct keys in the same order as (client, start,
    // index), sorted keys-only (one 64-bit compare per exchange) and unpacked after
    const bool pk = BIG_DS_PACKED && D <= 64 && NR < (1u << 26);
    auto rank_of = [&](uint32_t c) -> uint64_t {
      uint32_t lo = 0, hi = D;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (d_client[mid] < c) lo = mid + 1;
        else hi = mid;
      }
      return lo;
    };
    for (uint32_t j0 = t; j0 < NR; j0 += RB * NT) {
      uint32_t xi[RB], xs[RB], pi[RB], ps[RB];
#pragma unroll
      for (uint32_t q = 0; q < RB; q++) {
        const uint32_t j = j0 + q * NT;
        xi[q] = j < NR ? g_ri[j] : 0;
        xs[q] = j < NR ? g_rs[j] : 0;
        // lane 0 also builds the key of j - 1 (the previous lane's key belongs to another wave)
        const bool pv = lane == 0 && j > 0 && j <= NR;
        pi[q] = pv ? g_ri[j - 1] : 0;
        ps[q] = pv ? g_rs[j - 1] : 0;
      }
      uint32_t xt[RB], xc[RB], pt[RB], pc[RB];
#pragma unroll
      for (uint32_t q = 0; q < RB; q++) {
        const uint32_t j = j0 + q * NT;
        xt[q] = j < NR ? g_et[xi[q]] : 0;
        xc[q] = j < NR ? g_ec[xi[q]] : 0;
        const bool pv = lane == 0 && j > 0 && j <= NR;
        pt[q] = pv ? g_et[pi[q]] : 0;
        pc[q] = pv ? g_ec[pi[q]] : 0;
      }
#pragma unroll
      for (uint32_t q = 0; q < RB; q++) {
        const uint32_t j = j0 + q * NT;
        const bool live = xt[q] & 0x80000000u;
        const uint64_t key = !live ? ~0ull
                             : pk  ? (rank_of(xc[q]) << 58) | ((uint64_t)xs[q] << 26) | j
                                   : (((uint64_t)xc[q] << 32) | xs[q]);
        if (j < NR) {
          g_k0[j] = key;
          if (!pk) g_v0[j] = j;
          live_n += live;
        }
        const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)key, 1, 64);
        const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(key >> 32), 1, 64);
        uint64_t prev = ((uint64_t)hi << 32) | lo;
        if (lane == 0)
          prev = !(pt[q] & 0x80000000u) ? ~0ull
                 : pk ? (rank_of(pc[q]) << 58) | ((uint64_t)ps[q] << 26) | (j - 1)
                      : (((uint64_t)pc[q] << 32) | ps[q]);
        if (j < NR && j > 0 && prev > key) bad = 1;
      }
    }
    bscan_sum<NT>(live_n, ws, NL);
    const bool srt = __syncthreads_or(bad);
    if (!pk) {
      if (srt && wg_sort<NT>(m.k0, m.v0, m.k1, m.v1, NR, lscr)) {
        dkey = m.k1;
        dval = m.v1;
      }
    } else {
      const int w = srt ? wg_sort<NT, true>(m.k0, m.v0, m.k1, m.v1, NR, lscr) : 0;
      const uint64_t *src = w ? m.k1 : m.k0;
      uint64_t *dst = w ? m.k0 : m.k1;
      uint32_t *dv = w ? m.v0 : m.v1;
      for (uint32_t j = t; j < NL; j += NT) {
        const uint64_t k = src[j];
        dst[j] = ((uint64_t)d_client[k >> 58] << 32) | (uint32_t)(k >> 26);
        dv[j] = (uint32_t)k & 0x3FFFFFFu;
      }
      __syncthreads();
      dkey = dst;
      dval = dv;
    }
  }
  mark(11);
  uint64_t *dk = (uint64_t *)dkey; // the component starts are stashed in the keys' low halves
  // union pass 1: component heads (start after the running end of the client) and the
  // inclusive running end; pass 2: component starts, sizes, offsets, head prefix counts
  {
    uint32_t cE = 0;
    for (uint32_t base = 0; base < NL; base += NT) {
      const uint32_t j = base + t;
      const bool valid = j < NL;
      bool ch = false;
      uint32_t s0 = 0, e = 0;
      if (valid) {
        ch = j == 0 || (dkey[j] >> 32) != (dkey[j - 1] >> 32);
        s0 = (uint32_t)dkey[j];
        e = m.re[dval[j]];
      }
      uint32_t pf, pv;
      bscan_seg<NT, OpMax>(valid && ch, e, ws, pf, pv);
      const uint32_t before = ch ? 0 : (pf ? pv : (cE > pv ? cE : pv));
      const uint32_t run = ch ? e : (before > e ? before : e);
      if (valid) {
        m.chead[j] = ch ? 3u : (s0 > before ? 1u : 0u);
        m.cend[j] = run;
      }
      const uint32_t lastj = (NL - base < (uint32_t)NT ? NL - base : (uint32_t)NT) - 1;
      if (t == lastj) sc[0] = run;
      __syncthreads();
      cE = sc[0];
      __syncthreads();
    }
  }
  uint32_t ds_comp_total = 0;
  {
    uint32_t cS = 0, cO = 0, cP = 0; // carries: component start, byte offset, component heads
    for (uint32_t base = 0; base < NL; base += NT) {
      const uint32_t j = base + t;
      const bool valid = j < NL;
      const bool hh = valid && (m.chead[j] & 1);
      const uint32_t s0 = valid ? (uint32_t)dkey[j] : 0;
      uint32_t pf, pv;
      bscan_seg<NT, OpFirst>(hh, hh ? s0 : 0, ws, pf, pv);
      // OpFirst keeps the value of the first flagged lane of a run: the exclusive prefix's
      // component start is that of the last head before j
      uint32_t cs = hh ? s0 : (pf ? pv : cS);
      const bool tail = valid && (j + 1 == NL || (m.chead[j + 1] & 1));
      const uint32_t sz = tail ? varlen(cs) + varlen(m.cend[j] - cs) : 0;
      uint32_t TS, TP;
      const uint32_t pre = bscan_sum<NT>(sz, ws, TS);
      const uint32_t hp = bscan_sum<NT>(hh ? 1u : 0u, ws, TP);
      if (valid) {
        m.coff[j] = cO + pre;
        m.cpre[j] = cP + hp;
        if (tail) dk[j] = (dkey[j] & 0xFFFFFFFF00000000ull) | cs;
      }
      const uint32_t lastj = (NL - base < (uint32_t)NT ? NL - base : (uint32_t)NT) - 1;
      if (t == lastj) sc[0] = cs;
      __syncthreads();
      cS = sc[0];
      cO += TS;
      cP += TP;
      __syncthreads();
    }
    ds_comp_total = cO;
    if (t == 0) {
      m.coff[NL] = cO;
      m.cpre[NL] = cP;
    }
  }
  __syncthreads();
  mark(12);
  // per distinct client (rank r, ascending client): [a, b) of the sorted live ranges
  for (uint32_t r = t; r < D; r += NT) {
    const uint32_t c = d_client[r];
    uint32_t lo = 0, hi = NL;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) / 2;
      if ((uint32_t)(dkey[mid] >> 32) < c) lo = mid + 1;
      else hi = mid;
    }
    const uint32_t a = lo;
    hi = NL;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) / 2;
      if ((uint32_t)(dkey[mid] >> 32) <= c) lo = mid + 1;
      else hi = mid;
    }
    d_beg[r] = a;
    r_end[r] = lo;
    r_ncomp[r] = m.cpre[lo] - m.cpre[a];
  }
  __syncthreads();
  if (t == 0) { // header offsets in iteration order (D is small)
    uint32_t pos = varlen(D);
    for (uint32_t i = 0; i < D; i++) {
      const uint32_t r = d_ord[i];
      const uint32_t bytes = m.coff[r_end[r]] - m.coff[d_beg[r]];
      r_off[r] = pos;
      pos += varlen(d_client[r]) + varlen(r_ncomp[r]) + bytes;
    }
    sc[2] = pos;
  }
  __syncthreads();
  const uint32_t ds_size = sc[2];
  (void)ds_comp_total;
  const uint64_t total = blocks_size + ds_size;
  if (total > cap) {
    finish(1, 0, 0);
    return;
  }
  uint8_t *dso = out + blocks_size;
  if (t == 0) {
    Writer w{dso, 0};
    w_var(w, D);
  }
  for (uint32_t r = t; r < D; r += NT) {
    Writer w{dso, r_off[r]};
    w_var(w, d_client[r]);
    w_var(w, r_ncomp[r]);
  }
  for (uint32_t j = t; j < NL; j += NT) {
    const bool tail = j + 1 == NL || (m.chead[j + 1] & 1);
    if (!tail) continue;
    const uint32_t c = (uint32_t)(dkey[j] >> 32);
    uint32_t lo = 0, hi = D;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) / 2;
      if (d_client[mid] < c) lo = mid + 1;
      else hi = mid;
    }
    const uint32_t r = lo;
    Writer w{dso, r_off[r] + varlen(c) + varlen(r_ncomp[r]) + (m.coff[j] - m.coff[d_beg[r]])};
    const uint32_t cs = (uint32_t)dkey[j];
    w_var(w, cs);
    w_var(w, m.cend[j] - cs);
  }
  stamp(5);
  finish(0, 0, total);
}

// ------------------------------------------------------------------ launchers
void launch_big_count(const BatchIn &b, const FastOut &o, uint32_t *counts, uint64_t *need, uint32_t *n_big,
                      uint32_t n_list, hipStream_t s) {
  if (!b.n_docs || !n_list) return;
  hipLaunchKernelGGL((k_big_count<256>), dim3(n_list), dim3(256), 0, s, b, o.path, o.status, o.out_start,
                     o.out_len, counts, need, n_big, o.npath, (const uint32_t *)o.big_list);
}
void launch_big_merge(const BatchIn &b, const uint32_t *counts, const uint64_t *scr_off, uint32_t *scratch,
                      const FastOut &o, uint32_t n_list, hipStream_t s) {
  if (!b.n_docs || !n_list) return;
  // two 512-lane workgroups per CU (4 waves per SIMD at 128 VGPRs, 2 x 68 KB of LDS): twice the
  // documents in flight of one 1024-lane workgroup per CU (C4: tiled 9.05 -> 6.81 ms);
  // env YMERGE_BIG_NT=1024 selects the single-workgroup build (A/B)
  static const int nt = getenv("YMERGE_BIG_NT") ? atoi(getenv("YMERGE_BIG_NT")) : 512;
  static const uint32_t flags = (getenv("YMERGE_BIG_DSBM") && atoi(getenv("YMERGE_BIG_DSBM")) == 0) ? 1u : 0u;
  if (nt == 1024)
    hipLaunchKernelGGL((k_big_merge<1024, 4>), dim3(n_list), dim3(1024), 0, s, b, counts, scr_off, scratch, o, flags);
  else
    hipLaunchKernelGGL((k_big_merge<512, 4>), dim3(n_list), dim3(512), 0, s, b, counts, scr_off, scratch, o, flags);
}

} // namespace ym
