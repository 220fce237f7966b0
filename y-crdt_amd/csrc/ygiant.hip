// ygiant.hip — merge_updates_v1 of one very long single-client document across the whole GPU.
//
// A document of ~10^5 updates (the automerge-paper trace: 259,778 per-op updates) is a
// single unit of work for every per-document kernel: the tiled kernel runs it on one CU.  When
// the document is the shape of one author's log — every block and every DeleteSet entry of one
// client, the blocks contiguous in clock in update order, each block canonical — yrs' merge
// (update.rs:537-704) writes that client's blocks in update order behind one section header,
// and the DeleteSet union of one client's ranges (id_set.rs:129-164).  That output is built
// here by grid-wide kernels over the k_decode records, with no per-document serial phase:
//   k_gs_pre    lane per update: blocks / ranges / bytes / clock lengths, shape checks
//   (scans)     block and range counts, block bytes, clock lengths (k_scan)
//   k_gs_write  lane per update: the clock-contiguity check, block bytes copied to their
//               scanned offsets, deleted ranges set in a bitmap over the clock space
//   k_gs_runs   lane per bitmap word: run starts and ends (a run = one squashed DeleteSet range:
//               union of overlapping and adjacent ranges, as IdRange::squash merges them)
//   (scan)      run offsets
//   k_gs_comp   lane per word: the starts and ends of the runs in it, at their scanned ranks
//   k_gs_size   lane per run: length, varint bytes
//   (scan)      range byte offsets
//   k_gs_ds     lane per run: the (start, length) varints
//   k_gs_final  section header, DeleteSet header, length / status / path of the document.
// Documents outside the shape keep path 2 and go to the tiled kernel as before.
#include <algorithm>
#include "ycodec.h"
#include "ycopy.h"
#include "ykernels.h"

namespace ym {

enum : uint32_t {
  GS_BAD = 0, GS_CMIN, GS_CMAX, GS_MAXEND, GS_FIRST = 4 /* u64 at words 4-5 */, GS_NW = 6 /* bitmap words */,
  GS_K = 7 /* squashed ranges */, GS_MINST = 8 /* smallest range start: the bitmap's base (its word) */,
  GS_WORDS = 16
};
enum : uint32_t {
  GSB_SLOW = 1,      // an update k_decode did not decode (exact walk needed)
  GSB_BLOCK = 2,     // a block that is not copied verbatim (re-encoded / panics)
  GSB_DS = 4,        // a DeleteSet shape outside the path (several entries, empty range)
  GSB_GAP = 8,       // blocks not contiguous in clock in update order
  GSB_RANGE = 16     // a deleted range beyond the bitmap
};

__device__ __forceinline__ void gs_rec(const GsArgs &a, uint32_t i, uint32_t w[6]) {
  const uint2 *rp = (const uint2 *)(a.rec + (size_t)(a.u0 + i) * REC_WORDS);
  const uint2 x0 = rp[0], x1 = rp[1], x2 = rp[2];
  w[0] = x0.x;
  w[1] = x0.y;
  w[2] = x1.x;
  w[3] = x1.y;
  w[4] = x2.x;
  w[5] = x2.y;
}

// an update whose DeleteSet entry has more than GS_DSCOOP ranges may hand them to its
// workgroup (dfr returns true): one lane setting the 1,233 ranges of a `rustcode` update held
// k_gs_write 0.56 ms
constexpr uint32_t GS_DSCOOP = 32, GS_DSCOOP_N = 8;
// per-update blocks / ranges; calls blk(client, clock, len, pos, meta) and rng(client, s, e),
// or dfr(client, ranges, n) for a long range list (true: taken)
template <class FB, class FR, class FD>
__device__ __forceinline__ uint32_t gs_visit(const GsArgs &a, uint32_t i, FB blk, FR rng, FD dfr) {
  uint32_t w[6];
  gs_rec(a, i, w);
  if (w[0] & (REC_SLOW | REC_ORDER | 0xFF)) return GSB_SLOW; // (REC_ORDER: the exact engine)
  const uint32_t shape = (w[0] >> 10) & 3;
  if (shape == REC_BLOCK) {
    blk(w[1], w[2], w[3], w[4], w[5]);
  } else if (shape == REC_DS) {
    const uint32_t nr = (w[0] >> 12) & 3;
    if (nr > 0) rng(w[1], w[2], w[3]);
    if (nr > 1) rng(w[1], w[4], w[5]);
  } else if (shape == REC_COMPLEX) {
    if (!(w[0] & REC_OVF)) return GSB_SLOW;
    const uint32_t nb = w[1], ne = w[2], nr = w[3];
    if (ne > 1) return GSB_DS;
    const uint32_t *ov = a.ovf + w[4];
    for (uint32_t k = 0; k < nb; k++) blk(ov[5 * k], ov[5 * k + 1], ov[5 * k + 2], ov[5 * k + 3], ov[5 * k + 4]);
    const uint32_t *rv = ov + 5 * nb + 2 * ne;
    if (nr > GS_DSCOOP && dfr(ov[5 * nb], rv, nr)) return 0;
    for (uint32_t k = 0; k < nr; k++) rng(ov[5 * nb], rv[3 * k], rv[3 * k + 1]);
  }
  return 0;
}

__global__ void __launch_bounds__(256) k_gs_pre(GsArgs a) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  for (uint32_t j = i; j < a.nwords; j += gridDim.x * 256) a.bm[j] = 0; // (k_gs_write sets it)
  uint32_t nb = 0, nr = 0, bad = 0, cmin = 0xFFFFFFFFu, cmax = 0, maxend = 0, minst = 0xFFFFFFFFu;
  uint64_t bytes = 0, lens = 0, first = ~0ull;
  __shared__ uint32_t s_nd, s_dn[GS_DSCOOP_N];
  __shared__ uint64_t s_dp[GS_DSCOOP_N];
  if (threadIdx.x == 0) s_nd = 0;
  __syncthreads();
  if (i < a.U) bad |= gs_visit(
      a, i,
      [&](uint32_t c, uint32_t k, uint32_t len, uint32_t, uint32_t meta) {
        if (meta & 12) bad |= GSB_BLOCK;
        if (nb == 0) first = ((uint64_t)i << 32) | k;
        nb++;
        bytes += meta >> 8;
        lens += len;
        cmin = c < cmin ? c : cmin;
        cmax = c > cmax ? c : cmax;
      },
      [&](uint32_t c, uint32_t s, uint32_t e) {
        if (e <= s) bad |= GSB_DS;
        nr++;
        maxend = e > maxend ? e : maxend;
        minst = s < minst ? s : minst;
        cmin = c < cmin ? c : cmin;
        cmax = c > cmax ? c : cmax;
      },
      [&](uint32_t c, const uint32_t *rv, uint32_t n) { // the workgroup scans the ranges below
        const uint32_t q = atomicAdd(&s_nd, 1u);
        if (q >= GS_DSCOOP_N) return false;
        s_dp[q] = (uint64_t)rv;
        s_dn[q] = n;
        nr += n;
        cmin = c < cmin ? c : cmin;
        cmax = c > cmax ? c : cmax;
        return true;
      });
  if (i < a.U) {
    a.cnt[i] = nb | ((uint64_t)nr << 32);
    a.bl[i] = (bytes << 32) | lens;
  } // block bytes (< 2^31 per document) | clock lengths (< 2^32)
  __syncthreads();
  const uint32_t nd = s_nd < GS_DSCOOP_N ? s_nd : GS_DSCOOP_N;
  for (uint32_t e = 0; e < nd; e++) { // (folded into this thread's partials)
    const uint32_t *rv = (const uint32_t *)s_dp[e];
    for (uint32_t k = threadIdx.x; k < s_dn[e]; k += 256) {
      const uint32_t rs = rv[3 * k], re = rv[3 * k + 1];
      if (re <= rs) bad |= GSB_DS;
      maxend = re > maxend ? re : maxend;
      minst = rs < minst ? rs : minst;
    }
  }
  // workgroup partials (wave shuffles, then LDS), reduced by k_gs_reduce: atomics from every
  // wave on the same five words serialised at one L2 channel (165 us for the C1 trace)
  for (int o = 32; o > 0; o >>= 1) {
    bad |= __shfl_xor(bad, o, 64);
    const uint32_t c0 = __shfl_xor(cmin, o, 64), c1 = __shfl_xor(cmax, o, 64), m = __shfl_xor(maxend, o, 64);
    const uint32_t ms = __shfl_xor(minst, o, 64);
    cmin = c0 < cmin ? c0 : cmin;
    cmax = c1 > cmax ? c1 : cmax;
    maxend = m > maxend ? m : maxend;
    minst = ms < minst ? ms : minst;
    const uint64_t f = __shfl_xor(first, o, 64);
    first = f < first ? f : first;
  }
  __shared__ uint32_t part[4][7];
  const uint32_t wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[wv][0] = bad;
    part[wv][1] = cmin;
    part[wv][2] = cmax;
    part[wv][3] = maxend;
    part[wv][4] = (uint32_t)first;
    part[wv][5] = (uint32_t)(first >> 32);
    part[wv][6] = minst;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t q = 1; q < 4; q++) {
      bad |= part[q][0];
      cmin = part[q][1] < cmin ? part[q][1] : cmin;
      cmax = part[q][2] > cmax ? part[q][2] : cmax;
      maxend = part[q][3] > maxend ? part[q][3] : maxend;
      minst = part[q][6] < minst ? part[q][6] : minst;
      const uint64_t f = ((uint64_t)part[q][5] << 32) | part[q][4];
      first = f < first ? f : first;
    }
    uint32_t *gp = a.gp + 7 * blockIdx.x;
    gp[0] = bad;
    gp[1] = cmin;
    gp[2] = cmax;
    gp[3] = maxend;
    gp[4] = (uint32_t)first;
    gp[5] = (uint32_t)(first >> 32);
    gp[6] = minst;
  }
}

// one workgroup: the k_gs_pre partials -> the document's flags / client range / max range end /
// first block key
__global__ void __launch_bounds__(1024) k_gs_reduce(GsArgs a, uint32_t nparts) {
  uint32_t bad = 0, cmin = 0xFFFFFFFFu, cmax = 0, maxend = 0, minst = 0xFFFFFFFFu;
  uint64_t first = ~0ull;
  for (uint32_t q = threadIdx.x; q < nparts; q += 1024) {
    const uint32_t *gp = a.gp + 7 * q;
    bad |= gp[0];
    cmin = gp[1] < cmin ? gp[1] : cmin;
    cmax = gp[2] > cmax ? gp[2] : cmax;
    maxend = gp[3] > maxend ? gp[3] : maxend;
    minst = gp[6] < minst ? gp[6] : minst;
    const uint64_t f = ((uint64_t)gp[5] << 32) | gp[4];
    first = f < first ? f : first;
  }
  for (int o = 32; o > 0; o >>= 1) {
    bad |= __shfl_xor(bad, o, 64);
    const uint32_t c0 = __shfl_xor(cmin, o, 64), c1 = __shfl_xor(cmax, o, 64), m = __shfl_xor(maxend, o, 64);
    const uint32_t ms = __shfl_xor(minst, o, 64);
    cmin = c0 < cmin ? c0 : cmin;
    cmax = c1 > cmax ? c1 : cmax;
    maxend = m > maxend ? m : maxend;
    minst = ms < minst ? ms : minst;
    const uint64_t f = __shfl_xor(first, o, 64);
    first = f < first ? f : first;
  }
  __shared__ uint32_t part[16][7];
  const uint32_t wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[wv][0] = bad;
    part[wv][1] = cmin;
    part[wv][2] = cmax;
    part[wv][3] = maxend;
    part[wv][4] = (uint32_t)first;
    part[wv][5] = (uint32_t)(first >> 32);
    part[wv][6] = minst;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t q = 1; q < 16; q++) {
      bad |= part[q][0];
      cmin = part[q][1] < cmin ? part[q][1] : cmin;
      cmax = part[q][2] > cmax ? part[q][2] : cmax;
      maxend = part[q][3] > maxend ? part[q][3] : maxend;
      minst = part[q][6] < minst ? part[q][6] : minst;
      const uint64_t f = ((uint64_t)part[q][5] << 32) | part[q][4];
      first = f < first ? f : first;
    }
    a.g[GS_BAD] = bad;
    a.g[GS_CMIN] = cmin;
    a.g[GS_CMAX] = cmax;
    a.g[GS_MAXEND] = maxend;
    *(uint64_t *)(a.g + GS_FIRST) = first;
    a.g[GS_MINST] = minst == 0xFFFFFFFFu ? 0u : minst >> 5; // (word of the smallest start)
  }
}

// the document's output slot and its capacity (2 x its bytes + 64, as every path's slot)
__device__ __forceinline__ uint8_t *gs_out(const GsArgs &a) { return a.out + 2 * a.upd_off[a.u0] + 64ull * a.d; }
__device__ __forceinline__ uint64_t gs_cap(const GsArgs &a) {
  return 2 * (a.upd_off[a.u0 + a.U] - a.upd_off[a.u0]) + 64;
}

__device__ __forceinline__ uint32_t gs_hdr(const GsArgs &a) { // bytes of the one-section header
  const uint32_t nbt = (uint32_t)a.s_cnt[a.U];
  return varlen(1) + varlen(nbt) + varlen(a.g[GS_CMIN]) + varlen((uint32_t)*(const uint64_t *)(a.g + GS_FIRST));
}

// verbatim blocks of >= GS_COOP bytes are copied by the whole workgroup after its lanes' walks
constexpr uint32_t GS_COOP = 256, GS_COOP_N = 64;
// bits [s, e) of the deleted-clock bitmap (from the bitmap's base clock): the partial end
// words by atomicOr, the whole words between them directly (ranges over 64 words: queued for
// the workgroup's fill)
__device__ __forceinline__ void gs_set_range(const GsArgs &a, uint32_t base, uint32_t s, uint32_t e, uint32_t &bad,
                                             uint32_t &s_nr, uint32_t *s_r0, uint32_t *s_r1) {
  if (e - base > a.nbits) {
    bad |= GSB_RANGE;
    return;
  }
  s -= base;
  e -= base;
  const uint32_t w0 = s >> 5, w1 = (e - 1) >> 5;
  const uint32_t m0 = 0xFFFFFFFFu << (s & 31), m1 = 0xFFFFFFFFu >> (31 - ((e - 1) & 31));
  if (w0 == w1) {
    atomicOr(&a.bm[w0], m0 & m1);
  } else {
    atomicOr(&a.bm[w0], m0);
    uint32_t q = GS_COOP_N;
    if (w1 - w0 > 64) q = atomicAdd(&s_nr, 1u);
    if (q < GS_COOP_N) { // the workgroup fills the whole words after the walks
      s_r0[q] = w0 + 1;
      s_r1[q] = w1;
    } else {
      for (uint32_t z = w0 + 1; z < w1; z++) a.bm[z] = 0xFFFFFFFFu;
    }
    atomicOr(&a.bm[w1], m1);
  }
}
__device__ __forceinline__ void gs_write_lane(const GsArgs &a, uint32_t i, uint32_t &s_n, uint32_t *s_l, uint64_t *s_d,
                                              uint64_t *s_s, uint32_t &s_nr, uint32_t *s_r0, uint32_t *s_r1,
                                              uint32_t &s_nd, uint64_t *s_dp, uint32_t *s_dn);
__global__ void __launch_bounds__(256) k_gs_write(GsArgs a) {
  __shared__ uint32_t s_n, s_l[GS_COOP_N], s_nr, s_r0[GS_COOP_N], s_r1[GS_COOP_N];
  __shared__ uint64_t s_d[GS_COOP_N], s_s[GS_COOP_N];
  __shared__ uint32_t s_nd, s_dn[GS_DSCOOP_N];
  __shared__ uint64_t s_dp[GS_DSCOOP_N];
  if (threadIdx.x == 0) s_n = s_nr = s_nd = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < a.U) gs_write_lane(a, i, s_n, s_l, s_d, s_s, s_nr, s_r0, s_r1, s_nd, s_dp, s_dn);
  __syncthreads();
  const uint32_t nc = s_n < GS_COOP_N ? s_n : GS_COOP_N;
  for (uint32_t e = 0; e < nc; e++) copy_coop((uint8_t *)s_d[e], (const uint8_t *)s_s[e], s_l[e], threadIdx.x, 256);
  // long range lists handed over by the lanes, one range per thread
  const uint32_t nd = s_nd < GS_DSCOOP_N ? s_nd : GS_DSCOOP_N;
  if (nd) {
    const uint32_t base = 32 * a.g[GS_MINST];
    uint32_t bad = 0;
    for (uint32_t e = 0; e < nd; e++) {
      const uint32_t *rv = (const uint32_t *)s_dp[e];
      for (uint32_t k = threadIdx.x; k < s_dn[e]; k += 256) gs_set_range(a, base, rv[3 * k], rv[3 * k + 1], bad, s_nr, s_r0, s_r1);
    }
    if (bad) atomicOr(&a.g[GS_BAD], bad);
  }
  __syncthreads();
  // whole bitmap words of long deleted ranges (every bit set: plain stores are exact against
  // the other lanes' atomic ORs); one lane ORing a 60k-clock delete word by word took 0.5 ms
  const uint32_t nr = s_nr < GS_COOP_N ? s_nr : GS_COOP_N;
  for (uint32_t e = 0; e < nr; e++)
    for (uint32_t q = s_r0[e] + threadIdx.x; q < s_r1[e]; q += 256) a.bm[q] = 0xFFFFFFFFu;
}
__device__ __forceinline__ void gs_write_lane(const GsArgs &a, uint32_t i, uint32_t &s_n, uint32_t *s_l, uint64_t *s_d,
                                              uint64_t *s_s, uint32_t &s_nr, uint32_t *s_r0, uint32_t *s_r1,
                                              uint32_t &s_nd, uint64_t *s_dp, uint32_t *s_dn) {
  const uint32_t clock0 = (uint32_t)*(const uint64_t *)(a.g + GS_FIRST);
  uint64_t expect = clock0 + (a.s_bl[i] & 0xFFFFFFFFu);
  uint8_t *dst = gs_out(a) + gs_hdr(a) + (a.s_bl[i] >> 32);
  const uint8_t *src = a.bytes + a.upd_off[a.u0 + i];
  uint32_t bad = 0;
  // the bitmap covers clocks from the word of the smallest deleted clock on (a log whose clocks
  // start high -- the recent tail of a long-lived document -- does not need bits below it)
  const uint32_t base = 32 * a.g[GS_MINST];
  if (i == 0) { // bitmap words in use (the last one stays clear: run ends); over the buffer: bad
    const uint32_t nw = a.g[GS_MAXEND] > base ? (a.g[GS_MAXEND] - base) / 32 + 2 : 2u;
    a.g[GS_NW] = nw <= a.nwords ? nw : 0;
    if (nw > a.nwords) bad |= GSB_RANGE;
  }
  gs_visit(
      a, i,
      [&](uint32_t, uint32_t k, uint32_t len, uint32_t pos, uint32_t meta) {
        if (k != expect) bad |= GSB_GAP;
        expect += len;
        const uint32_t n = meta >> 8;
        uint32_t q = GS_COOP_N;
        if (n >= GS_COOP) q = atomicAdd(&s_n, 1u);
        if (q < GS_COOP_N) {
          s_d[q] = (uint64_t)dst;
          s_s[q] = (uint64_t)(src + pos);
          s_l[q] = n;
        } else {
          Writer w{dst, 0}; // (16-byte load groups: a byte loop waits one load latency per byte)
          w.bytes(src + pos, n);
        }
        dst += n;
      },
      [&](uint32_t, uint32_t s, uint32_t e) { gs_set_range(a, base, s, e, bad, s_nr, s_r0, s_r1); },
      [&](uint32_t, const uint32_t *rv, uint32_t n) {
        const uint32_t q = atomicAdd(&s_nd, 1u);
        if (q >= GS_DSCOOP_N) return false;
        s_dp[q] = (uint64_t)rv;
        s_dn[q] = n;
        return true;
      });
  if (bad) atomicOr(&a.g[GS_BAD], bad);
}

__device__ __forceinline__ uint32_t gs_starts(const GsArgs &a, uint32_t j) {
  const uint32_t w = a.bm[j], prev = j ? a.bm[j - 1] >> 31 : 0u;
  return w & ~((w << 1) | prev);
}
// last bits of runs (the bitmap's last word in use is clear, so every run ends)
__device__ __forceinline__ uint32_t gs_ends(const GsArgs &a, uint32_t j) {
  const uint32_t w = a.bm[j], next = a.bm[j + 1] & 1u;
  return w & ~((w >> 1) | (next << 31));
}

// kernels over the bitmap / the runs: grid-stride up to the counts on the device (the grid is
// sized for the buffers' capacity, so no host round trip sits between the stages)
__global__ void __launch_bounds__(256) k_gs_runs(GsArgs a) {
  const uint32_t nw = a.g[GS_NW];
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < nw; j += gridDim.x * 256)
    a.w_cnt[j] = a.g[GS_BAD] || j + 1 >= nw ? 0 : __popc(gs_starts(a, j)) | ((uint64_t)__popc(gs_ends(a, j)) << 32);
}

// run k: its first bit from the k-th start, its end from the k-th end (scanned per word), so no
// lane walks a long run word by word
__global__ void __launch_bounds__(256) k_gs_comp(GsArgs a) {
  const uint32_t nw = a.g[GS_NW];
  if (a.g[GS_BAD]) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // (32-bit halves: this hipcc miscompiled the 64-bit uniform compare feeding a select,
    // testing SCC after a VALU compare that set VCC)
    const uint32_t kl = (uint32_t)a.w_scan[nw];
    const uint32_t over = kl > a.kcap;
    a.g[GS_K] = kl & (over - 1u);
    if (over) atomicOr(&a.g[GS_BAD], GSB_RANGE);
  }
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j + 1 < nw; j += gridDim.x * 256) {
    const uint64_t sc = a.w_scan[j];
    uint32_t ks = (uint32_t)sc, ke = (uint32_t)(sc >> 32);
    uint32_t st = gs_starts(a, j), en = gs_ends(a, j);
    if (ks + __popc(st) > a.kcap || ke + __popc(en) > a.kcap) continue; // (then the document is bad)
    const uint32_t base = 32 * a.g[GS_MINST];
    while (st) {
      a.k_start[ks++] = base + 32 * j + __builtin_ctz(st);
      st &= st - 1;
    }
    while (en) {
      a.k_len[ke++] = base + 32 * j + __builtin_ctz(en) + 1; // end (exclusive) for now: k_gs_size subtracts
      en &= en - 1;
    }
  }
}

// per run: length and varint bytes
__global__ void __launch_bounds__(256) k_gs_size(GsArgs a) {
  if (a.g[GS_BAD]) return;
  const uint32_t K = a.g[GS_K];
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < K; k += gridDim.x * 256) {
    const uint32_t s = a.k_start[k], n = a.k_len[k] - s;
    a.k_len[k] = n;
    a.k_size[k] = varlen(s) + varlen(n);
  }
}

__device__ __forceinline__ uint64_t gs_ds_base(const GsArgs &a) {
  const uint32_t K = a.g[GS_K];
  return gs_hdr(a) + (a.s_bl[a.U] >> 32) + (K ? varlen(1) + varlen(a.g[GS_CMIN]) + varlen(K) : varlen(0));
}

__global__ void __launch_bounds__(256) k_gs_ds(GsArgs a) {
  if (a.g[GS_BAD]) return;
  const uint32_t K = a.g[GS_K];
  uint8_t *base = gs_out(a) + gs_ds_base(a);
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < K; k += gridDim.x * 256) {
    Writer w{base + a.k_off[k], 0};
    w_var(w, a.k_start[k]);
    w_var(w, a.k_len[k]);
  }
}

__global__ void k_gs_final(GsArgs a, FastOut o) {
  if (threadIdx.x) return;
  const uint32_t K = a.g[GS_BAD] ? 0 : a.g[GS_K];
  const uint64_t total = a.g[GS_BAD] ? 0 : gs_ds_base(a) + a.k_off[K];
  o.out_start[a.d] = 2 * a.upd_off[a.u0] + 64ull * a.d;
  if (a.g[GS_BAD] || total > gs_cap(a)) { // not the shape after all: the tiled kernel writes it
    o.path[a.d] = 2;
    return;
  }
  Writer w{gs_out(a), 0};
  w_var(w, 1);
  w_var(w, (uint32_t)a.s_cnt[a.U]);
  w_var(w, a.g[GS_CMIN]);
  w_var(w, (uint32_t)*(const uint64_t *)(a.g + GS_FIRST));
  Writer v{gs_out(a) + gs_hdr(a) + (a.s_bl[a.U] >> 32), 0};
  if (K) {
    w_var(v, 1);
    w_var(v, a.g[GS_CMIN]);
    w_var(v, K);
  } else {
    w_var(v, 0);
  }
  o.out_len[a.d] = total;
  o.status[a.d] = 0;
  o.path[a.d] = 0; // written: the tiled kernel skips it
  atomicAdd(&o.npath[14], 1u);
}

// documents the tiled kernel would take (path 2) with at least min_u updates: list[0] =
// count, then (document, updates, ranges, first update, first byte, bytes) for up to GS_LIST
__global__ void k_gs_find(BatchIn b, uint8_t *path, uint32_t min_u, uint64_t *list) {
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d >= b.n_docs || path[d] != 2) return;
  const uint64_t u0 = b.doc_upd[d], u1 = b.doc_upd[d + 1];
  if (u1 - u0 < min_u || u1 - u0 >= (1ull << 31)) return;
  const uint64_t k = atomicAdd((unsigned long long *)&list[0], 1ull);
  if (k < GS_LIST) {
    path[d] = GS_PATH; // k_big_count skips it; k_gs_final sets 0 (written) or 2 (tiled kernel)
    uint64_t *e = list + 1 + 6 * k;
    e[0] = d;
    e[1] = u1 - u0;
    e[2] = 0;
    e[3] = u0;
    e[4] = b.upd_off[u0];
    e[5] = b.upd_off[u1] - b.upd_off[u0];
  }
}

void launch_gs_find(const BatchIn &b, uint8_t *path, uint32_t min_u, uint64_t *list, hipStream_t s) {
  if (!b.n_docs) return;
  hipLaunchKernelGGL(k_gs_find, dim3((b.n_docs + 255) / 256), dim3(256), 0, s, b, path, min_u, list);
}
void launch_gs_pre(const GsArgs &a, hipStream_t s) {
  const uint32_t nb = (a.U + 255) / 256;
  hipLaunchKernelGGL(k_gs_pre, dim3(nb), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_gs_reduce, dim3(1), dim3(1024), 0, s, a, nb);
}
void launch_gs_rest(const GsArgs &a, const FastOut &o, uint64_t *scan_tmp, hipStream_t s) {
  const uint32_t gw = std::min<uint32_t>((a.nwords + 255) / 256, 1024u), gk = std::min<uint32_t>((a.kcap + 255) / 256, 1024u);
  hipLaunchKernelGGL(k_gs_write, dim3((a.U + 255) / 256), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_gs_runs, dim3(gw), dim3(256), 0, s, a);
  launch_scan_u64(a.w_cnt, a.w_scan, a.nwords, scan_tmp, s, a.g + GS_NW);
  hipLaunchKernelGGL(k_gs_comp, dim3(gw), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_gs_size, dim3(gk), dim3(256), 0, s, a);
  launch_scan_u64(a.k_size, a.k_off, a.kcap, scan_tmp, s, a.g + GS_K);
  hipLaunchKernelGGL(k_gs_ds, dim3(gk), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_gs_final, dim3(1), dim3(64), 0, s, a, o);
}

} // namespace ym
