// ylwin.h -- LDS window cursor for one long update walked by a whole wavefront in lockstep.
//
// An update far larger than any per-update stage (the reference's b4-update.bin: 400,972 bytes,
// 12,387 blocks in one update) was walked by one lane through the 64-byte register window
// of ywin.h, ~700 cycles per byte (one memory round trip per block and a select tree per byte).
// Here the 64 lanes of a wave walk the same update together: the state machine is the same for
// every lane (same bytes, same branches), so the wave behaves like one walker, while every
// refill of the window is a cooperative copy -- lane k loads the 16-byte chunks k, k + 64, ...
// of the next LW_BYTES, all in flight at once -- and every byte read is an LDS read.
// Same interface as WCur (wc_byte / wc_ensure / wc_skip, fields p, n, i), so smwalk_update
// (ysm.h) runs on it unchanged.
#pragma once
#include "ycodec.h"

namespace ym {

constexpr uint32_t LW_BYTES = 16384; // window bytes (LDS of the calling wave)

struct LWin {
  const uint8_t *p; // stream start (global memory)
  uint32_t n, i;    // length, position
  uint32_t *w;      // LDS window [LW_BYTES / 4]
  uint64_t wa;      // absolute address of the window's first byte (16-byte aligned)
  uint32_t lane;
};

YM_INLINE void lw_init(LWin &c, const uint8_t *p, uint32_t n, uint32_t *w) {
  c.p = p;
  c.n = n;
  c.i = 0;
  c.w = w;
  c.wa = ~0ull << 20; // forces a load on first access
  c.lane = threadIdx.x & 63;
}

// window = the 16-byte chunks from a (aligned) that hold stream bytes, at most LW_BYTES
YM_INLINE void lw_load(LWin &c, uint64_t a) {
  const uint64_t end = (uint64_t)(c.p + c.n);
  const uint32_t nch = (uint32_t)((end - a + 15) >> 4) < LW_BYTES / 16 ? (uint32_t)((end - a + 15) >> 4) : LW_BYTES / 16;
  __builtin_amdgcn_wave_barrier(); // every lane's reads of the old window are done
  const uint4 *q = (const uint4 *)a;
  uint4 *dst = (uint4 *)c.w;
  for (uint32_t k = c.lane; k < nch; k += 64) dst[k] = q[k];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  c.wa = a;
}

YM_INLINE uint32_t wc_byte(LWin &c, uint32_t pos) {
  const uint64_t a = (uint64_t)(c.p + pos);
  if (a < c.wa || a >= c.wa + LW_BYTES) lw_load(c, a & ~15ull);
  const uint32_t off = (uint32_t)(a - c.wa);
  return (c.w[off >> 2] >> ((off & 3) * 8)) & 0xFF;
}
YM_INLINE void wc_ensure(LWin &c, uint32_t need) {
  const uint64_t a = (uint64_t)(c.p + c.i), lim = (uint64_t)(c.p + c.n);
  if (a >= lim) return;
  const uint64_t want = a + need < lim ? a + need : lim;
  if (a < c.wa || want > c.wa + LW_BYTES) lw_load(c, a & ~15ull);
}
YM_INLINE int wc_skip(LWin &c, uint64_t len) {
  if (len > (uint64_t)(c.n - c.i)) return E_EOS;
  c.i += (uint32_t)len;
  return 0;
}

} // namespace ym
