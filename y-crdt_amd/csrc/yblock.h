// yblock.h — workgroup-wide primitives and decode sinks shared by the one-workgroup-
// per-document merge kernels (ymerge_fast.hip: LDS-resident documents; ymerge_big.hip:
// documents above the LDS capacities, SoA in HBM scratch, processed in tiles).
#pragma once
#include "ycodec.h"
#include "ykernels.h"
#include "ywalk.h"
#include "ysm.h"

namespace ym {

__host__ __device__ inline uint32_t pow2ceil(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// ------------------------------------------------------------------ block-wide helpers
template <int NT> struct Blk {
  static constexpr int NW = NT / 64;
};

// exclusive sum over per-lane values; returns the lane's exclusive prefix, *total = sum
template <int NT> __device__ __forceinline__ uint32_t bscan_sum(uint32_t v, uint32_t *ws, uint32_t &total) {
  uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < NT / 64; i++) {
      uint32_t s = ws[i];
      ws[i] = acc;
      acc += s;
    }
    ws[NT / 64] = acc;
  }
  __syncthreads();
  uint32_t r = ws[w] + x - v;
  total = ws[NT / 64];
  __syncthreads();
  return r;
}

template <int NT> __device__ __forceinline__ uint64_t bscan_sum64(uint64_t v, uint64_t *ws64, uint64_t &total) {
  uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) ws64[w] = x;
  __syncthreads();
  if (t == 0) {
    uint64_t acc = 0;
    for (int i = 0; i < NT / 64; i++) {
      uint64_t s = ws64[i];
      ws64[i] = acc;
      acc += s;
    }
    ws64[NT / 64] = acc;
  }
  __syncthreads();
  uint64_t r = ws64[w] + x - v;
  total = ws64[NT / 64];
  __syncthreads();
  return r;
}

__device__ __forceinline__ uint32_t mix32(uint32_t c) { return c * 0x9E3779B9u; }

// segmented scan pair: (flag, value); (f1,v1)+(f2,v2) = (f1|f2, f2 ? v2 : op(v1,v2))
struct OpMax {
  __device__ static uint32_t f(uint32_t a, uint32_t b) { return a > b ? a : b; }
};
struct OpSum {
  __device__ static uint32_t f(uint32_t a, uint32_t b) { return a + b; }
};
struct OpFirst {
  __device__ static uint32_t f(uint32_t a, uint32_t) { return a; }
};
// Exclusive segmented scan of the per-lane aggregate (flag, v): returns (pf, pv) = combination
// of all lanes before this lane (pf = any head before in ... ), over the whole workgroup.
template <int NT, class Op>
__device__ __forceinline__ void bscan_seg(uint32_t f, uint32_t v, uint32_t *ws, uint32_t &pf, uint32_t &pv) {
  uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t xf = f, xv = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t yf = __shfl_up(xf, o, 64), yv = __shfl_up(xv, o, 64);
    if (lane >= (uint32_t)o) {
      xv = xf ? xv : Op::f(yv, xv);
      xf = xf | yf;
    }
  }
  // exclusive within wave
  uint32_t ef = __shfl_up(xf, 1, 64), ev = __shfl_up(xv, 1, 64);
  if (lane == 0) {
    ef = 0;
    ev = 0;
  }
  if (lane == 63) {
    ws[2 * w] = xf;
    ws[2 * w + 1] = xv;
  }
  __syncthreads();
  if (t == 0) {
    uint32_t af = 0, av = 0;
    for (int i = 0; i < NT / 64; i++) {
      uint32_t sf = ws[2 * i], sv = ws[2 * i + 1];
      ws[2 * i] = af;
      ws[2 * i + 1] = av;
      av = sf ? sv : Op::f(av, sv);
      af |= sf;
    }
  }
  __syncthreads();
  uint32_t wf = ws[2 * w], wv = ws[2 * w + 1];
  __syncthreads();
  // combine wave prefix (wf,wv) with in-wave exclusive (ef,ev)
  if (lane == 0) {
    pf = wf;
    pv = wv;
  } else {
    pv = ef ? ev : Op::f(wv, ev);
    pf = wf | ef;
  }
}

// bitonic sort of (key64, val32) pairs, n a power of two, composite order (key, val)
// Ascending bitonic sort of one u64 per lane across a wavefront (registers and lane
// shuffles, no LDS, no barrier); pad unused lanes with ~0.
YM_INLINE uint64_t wave_bitonic64(uint64_t x, uint32_t lane) {
#pragma unroll
  for (uint32_t size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)x, stride, 64), hi = __shfl_xor((uint32_t)(x >> 32), stride, 64);
      const uint64_t y = ((uint64_t)hi << 32) | lo;
      const bool take_min = ((lane & stride) == 0) == ((lane & size) == 0);
      x = take_min ? (x < y ? x : y) : (x < y ? y : x);
    }
  }
  return x;
}

template <int NT> YM_INLINE void bitonic(uint64_t *k, uint32_t *v, uint32_t n) {
  for (uint32_t size = 2; size <= n; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = threadIdx.x; i < n / 2; i += NT) {
        uint32_t lo = 2 * i - (i & (stride - 1));
        uint32_t hi = lo + stride;
        bool up = ((lo & size) == 0);
        uint64_t a = k[lo], b = k[hi];
        uint32_t va = v[lo], vb = v[hi];
        bool gt = a > b || (a == b && va > vb);
        if (gt == up) {
          k[lo] = b;
          k[hi] = a;
          v[lo] = vb;
          v[hi] = va;
        }
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------ walk sinks
// One walk per update.  The common shapes (<= 1 block, <= 1 DeleteSet entry with <= 2
// ranges) are kept in registers until the round's scan places them; any other update
// is re-walked once by FastFill at its scanned positions.
// TRACK: the section-order check (REC_ORDER); k_decode's fast walk leaves it to the second walk
// of its multi-record updates (OvfFill), which keeps its own walk within 64 VGPRs
template <bool TRACK> struct RegSinkT {
  uint32_t nb, ne, nr;
  bool unsupported, big_ds;
  bool misorder = false;                            // REC_ORDER
  uint32_t last_cl = 0xFFFFFFFFu;                   // (a first section of client 2^32 - 1 is flagged too)
  uint32_t b_client, b_clock, b_len, b_pos, b_meta; // first block
  uint32_t e_client;                                // first DeleteSet entry
  uint32_t r0s, r0e, r1s, r1e;                      // its first two ranges
  const uint8_t *doc;
  uint32_t doc_len, ubase;
  YM_INLINE void on_section(uint32_t client) {
    if (TRACK) {
      misorder |= client >= last_cl;
      last_cl = client;
    }
  }
  YM_INLINE int on_block(uint32_t client, uint32_t clock, const BlockInfo &bi, uint32_t bpos, uint32_t blen) {
    if (bi.unsupported) unsupported = true;
    if (bi.kind == BK_SKIP) return 0;
    if (nb == 0) {
      b_client = client;
      b_clock = clock;
      b_len = bi.len;
      b_pos = ubase + bpos;
      b_meta = (uint32_t)bi.kind | (bi.reenc ? 4u : 0u) | (bi.enc_panic ? 8u : 0u) | (blen << 8);
    }
    nb++;
    return 0;
  }
  YM_INLINE int on_ds_begin(uint32_t nds) {
    if (nds > DS_SMALL) big_ds = true; // table emulation beyond 16 buckets: exact engine
    return 0;
  }
  YM_INLINE int on_ds_entry(uint32_t client, uint32_t) {
    if (ne == 0) e_client = client;
    ne++;
    return 0;
  }
  YM_INLINE void on_ds_range(uint32_t s0, uint32_t e0) {
    if (nr == 0) {
      r0s = s0;
      r0e = e0;
    } else if (nr == 1) {
      r1s = s0;
      r1e = e0;
    }
    nr++;
  }
  YM_INLINE int on_ds_done() { return 0; }
};
using RegSink = RegSinkT<true>;

struct FastFill {
  uint32_t *bc, *bk, *bl, *bp, *bm, *ec, *et, *rs, *re, *ri;
  uint32_t upd, ubase; // update index, byte offset of update within doc
  uint32_t nb, ne, nr, ebase;
  YM_INLINE void on_section(uint32_t) {}
  YM_INLINE int on_block(uint32_t client, uint32_t clock, const BlockInfo &bi, uint32_t bpos, uint32_t blen) {
    if (bi.kind == BK_SKIP) return 0;
    bc[nb] = client;
    bk[nb] = clock;
    bl[nb] = bi.len;
    bp[nb] = ubase + bpos;
    bm[nb] = (uint32_t)bi.kind | (bi.reenc ? 4u : 0u) | (bi.enc_panic ? 8u : 0u) | (blen << 8);
    nb++;
    return 0;
  }
  YM_INLINE int on_ds_begin(uint32_t) {
    ebase = ne;
    return 0;
  }
  YM_INLINE int on_ds_entry(uint32_t client, uint32_t) {
    ec[ne] = client;
    et[ne] = 0x80000000u | (upd << 8);
    ne++;
    return 0;
  }
  YM_INLINE void on_ds_range(uint32_t s, uint32_t e) {
    rs[nr] = s;
    re[nr] = e;
    ri[nr] = ne - 1;
    nr++;
  }
  YM_INLINE int on_ds_done() {
    const uint32_t n = ne - ebase;
    if (n >= 2) ds_order_packed(ec + ebase, n, et + ebase, upd << 8); // (n <= DS_SMALL: else exact engine)
    return 0;
  }
};

// Writes one multi-record update (REC_COMPLEX) into its workgroup's overflow words:
// [blocks: 5 words each (client, clock, length, position in update, meta)]
// [entry clients] [entry table codes] [ranges: 3 words each (start, end, entry index
// within the update)].  The table code is the entry's iteration position in the update's
// DeleteSet HashMap | 0x80000000, or 0 if a later entry of the same client replaced it
// (ds_order_packed, computed here at k_decode's occupancy rather than by one lane of the
// merge workgroup).
struct OvfFill {
  uint32_t *ov;
  uint32_t NBt, NEt; // totals of this update (RegSink pass)
  uint32_t nb, ne, nr;
  bool on = true; // writes (a wave walking one update in lockstep: lane 0 only)
  bool misorder = false; // REC_ORDER (RegSinkT)
  uint32_t last_cl = 0xFFFFFFFFu;
  YM_INLINE void on_section(uint32_t client) {
    misorder |= client >= last_cl;
    last_cl = client;
  }
  YM_INLINE int on_block(uint32_t client, uint32_t clock, const BlockInfo &bi, uint32_t bpos, uint32_t blen) {
    if (bi.kind == BK_SKIP) return 0;
    if (on) {
      uint32_t *w = ov + 5 * nb;
      w[0] = client;
      w[1] = clock;
      w[2] = bi.len;
      w[3] = bpos;
      w[4] = (uint32_t)bi.kind | (bi.reenc ? 4u : 0u) | (bi.enc_panic ? 8u : 0u) | (blen << 8);
    }
    nb++;
    return 0;
  }
  YM_INLINE int on_ds_begin(uint32_t) { return 0; }
  YM_INLINE int on_ds_entry(uint32_t client, uint32_t) {
    if (on) ov[5 * NBt + ne] = client;
    ne++;
    return 0;
  }
  YM_INLINE void on_ds_range(uint32_t s0, uint32_t e0) {
    if (on) {
      uint32_t *w = ov + 5 * NBt + 2 * NEt + 3 * nr;
      w[0] = s0;
      w[1] = e0;
      w[2] = ne - 1;
    }
    nr++;
  }
  YM_INLINE int on_ds_done() {
    uint32_t *cl = ov + 5 * NBt;
    if (!on) return 0;
    if (ne == 1) cl[1] = 0x80000000u;
    else if (ne >= 2) ds_order_packed(cl, ne, cl + ne, 0);
    return 0;
  }
};

// sink -> record (ykernels.h REC_*); positions stay relative to the update
template <bool T>
YM_INLINE void rec_pack(const RegSinkT<T> &s, int e, uint32_t &w0, uint32_t &w1, uint32_t &w2, uint32_t &w3, uint32_t &w4,
                        uint32_t &w5) {
  w0 = (uint32_t)e & 0xFF;
  w1 = w2 = w3 = w4 = w5 = 0;
  if (s.unsupported) w0 |= REC_UNSUP;
  if (s.big_ds) w0 |= REC_BIGDS;
  if (s.misorder) w0 |= REC_ORDER;
  if (e) return;
  if (s.nb == 1 && s.ne == 0) {
    w0 |= REC_BLOCK << 10;
    w1 = s.b_client;
    w2 = s.b_clock;
    w3 = s.b_len;
    w4 = s.b_pos;
    w5 = s.b_meta;
  } else if (s.nb == 0 && s.ne == 1 && s.nr <= 2) {
    w0 |= (REC_DS << 10) | (s.nr << 12);
    w1 = s.e_client;
    w2 = s.r0s;
    w3 = s.r0e;
    w4 = s.r1s;
    w5 = s.r1e;
  } else if (s.nb || s.ne) {
    w0 |= REC_COMPLEX << 10;
    w1 = s.nb;
    w2 = s.ne;
    w3 = s.nr;
  }
}

// canonical encoded size of a kept block (bm: kind | reenc 4 | panic 8 | input bytes << 8)
__device__ __forceinline__ uint32_t canon_size(const uint8_t *doc, uint32_t doc_len, uint32_t pos, uint32_t client,
                                               uint32_t clock, uint32_t len, uint32_t meta) {
  if (!(meta & 4) || (meta & 8)) return meta >> 8;
  Counter cn;
  emit_block(doc, doc_len, pos, client, clock, len, 0, cn);
  return (uint32_t)cn.n;
}

// Cold paths out of line (they keep the merge kernels' register allocation small):
// the exact walk of one update over HBM into a record / into its scanned positions.
__device__ __noinline__ int walk_record_hbm(const uint8_t *p, uint32_t n, uint32_t *w) {
  RegSink s;
  s.nb = s.ne = s.nr = 0;
  s.unsupported = s.big_ds = false;
  s.ubase = 0;
  WCur c;
  wc_init(c, p, n);
  const int e = smwalk_update(c, s);
  rec_pack(s, e, w[0], w[1], w[2], w[3], w[4], w[5]);
  return e;
}
__device__ __noinline__ void fill_hbm(const uint8_t *p, uint32_t n, FastFill *f) {
  WCur c;
  wc_init(c, p, n);
  smwalk_update(c, *f);
}

} // namespace ym
