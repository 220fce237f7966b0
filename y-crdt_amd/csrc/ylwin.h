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
// the window is addressed as LDS (ds_read / ds_write): through a generic pointer every byte
// read would be a flat access, which takes the vector-memory path
typedef __attribute__((address_space(3))) uint32_t lds_u32;

struct LWin {
  const uint8_t *p; // stream start (global memory)
  uint32_t n, i;    // length, position
  lds_u32 *w;       // LDS window [LW_BYTES / 4]
  uint64_t wa;      // absolute address of the window's first byte (16-byte aligned)
  uint32_t lane;
};

YM_INLINE void lw_init(LWin &c, const uint8_t *p, uint32_t n, lds_u32 *w) {
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
  for (uint32_t k = c.lane; k < nch; k += 64) {
    const uint4 v = q[k];
    c.w[4 * k] = v.x;
    c.w[4 * k + 1] = v.y;
    c.w[4 * k + 2] = v.z;
    c.w[4 * k + 3] = v.w;
  }
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
// A varint / raw byte from 16 window bytes at once (two ds_read_b64 instead of a dependent
// LDS read per byte); the general path near the window's or the stream's end.
YM_INLINE int wc_read(LWin &c, bool raw, uint32_t &v, bool &canon) {
  const uint64_t a = (uint64_t)(c.p + c.i);
  if (c.i + 12 <= c.n && a >= c.wa && a + 16 <= c.wa + LW_BYTES) {
    const uint32_t off = (uint32_t)(a - c.wa), q = off >> 2, sh = (off & 3) * 8;
    const uint64_t x01 = ((uint64_t)c.w[q + 1] << 32) | c.w[q], x23 = ((uint64_t)c.w[q + 3] << 32) | c.w[q + 2];
    const uint64_t lo = sh ? (x01 >> sh) | (x23 << (64 - sh)) : x01; // stream bytes 0..7
    const uint32_t hi = (uint32_t)(x23 >> sh);                         // stream bytes 8..11
    if (raw) {
      v = (uint32_t)lo & 0xFF;
      c.i++;
      return 0;
    }
    const uint64_t stop0 = ~lo & 0x8080808080808080ull;
    const uint32_t stop1 = ~hi & 0x00808080u;
    if (!stop0 && !stop1) return E_VARINT; // no terminator in 11 bytes
    const uint32_t n = stop0 ? ((uint32_t)__builtin_ctzll(stop0) >> 3) + 1 : ((uint32_t)__builtin_ctz(stop1) >> 3) + 9;
    uint32_t x = 0;
#pragma unroll
    for (uint32_t k = 0; k < 11; k++) {
      const uint32_t byte = k < 8 ? (uint32_t)(lo >> (8 * k)) & 0xFF : (hi >> (8 * (k - 8))) & 0xFF;
      if (k < n) x |= (byte & 0x7f) << ((7 * k) & 31);
    }
    const uint32_t last = n <= 8 ? (uint32_t)(lo >> (8 * (n - 1))) & 0xFF : (hi >> (8 * (n - 9))) & 0xFF;
    v = x;
    canon = n == varlen(x) && (n != 5 || last < 16);
    c.i += n;
    return 0;
  }
  uint32_t sh = 0, nbytes = 0, b = 0;
  v = 0;
  for (;;) {
    if (c.i >= c.n) return E_EOS;
    b = wc_byte(c, c.i++);
    if (raw) {
      v = b;
      return 0;
    }
    v |= (b & 0x7f) << (sh & 31);
    sh += 7;
    nbytes++;
    if (b < 0x80) break;
    if (sh > 70) return E_VARINT;
  }
  canon = nbytes == varlen(v) && (nbytes != 5 || b < 16);
  return 0;
}
// OR of the bytes [s0, s0 + n) dword-wise when they are in the window
YM_INLINE uint32_t wc_or(LWin &c, uint32_t s0, uint32_t n) {
  const uint64_t a = (uint64_t)(c.p + s0);
  if (n && a >= c.wa && a + n + 4 <= c.wa + LW_BYTES) {
    const uint32_t o0 = (uint32_t)(a - c.wa), e0 = o0 + n, q0 = o0 >> 2, q1 = (e0 - 1) >> 2;
    uint32_t hi = 0;
    for (uint32_t q = q0; q <= q1; q++) {
      uint32_t x = c.w[q];
      if (q == q0) x &= 0xFFFFFFFFu << (8 * (o0 & 3));
      if (q == q1 && (e0 & 3)) x &= 0xFFFFFFFFu >> (8 * (4 - (e0 & 3)));
      hi |= x;
    }
    return (hi | (hi >> 8) | (hi >> 16) | (hi >> 24)) & 0xFF;
  }
  uint32_t hi = 0;
  for (uint32_t q = 0; q < n; q++) hi |= wc_byte(c, s0 + q);
  return hi;
}
YM_INLINE int wc_skip(LWin &c, uint64_t len) {
  if (len > (uint64_t)(c.n - c.i)) return E_EOS;
  c.i += (uint32_t)len;
  return 0;
}

} // namespace ym
