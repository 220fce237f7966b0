// ywave.h — wavefront primitives shared by the one-wavefront-per-document kernels
// (ymerge_lean.hip: k_lean; ydiff.hip: k_plan_wave): lane masks, readlane / shuffles pinned
// to where they are computed, DPP inclusive sums, and the branch-free LEB128 read of staged
// LDS words.
#pragma once
#include "ycodec.h"

namespace ym {

// ------------------------------------------------------------------ wave primitives
YM_INLINE void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
YM_INLINE uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
YM_INLINE uint32_t rdlane(uint32_t x, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane(x, l); }
// (the builtin returns int: each half is widened as unsigned, or a low word >= 2^31 would
// sign-extend into the high word)
YM_INLINE uint64_t rdlane64(uint64_t x, uint32_t l) {
  return ((uint64_t)rdlane((uint32_t)(x >> 32), l) << 32) | (uint64_t)rdlane((uint32_t)x, l);
}
// Cross-lane results are pinned where they are computed: the backend may otherwise sink a
// ds_bpermute into a branch whose exec mask excludes its source lanes (observed: the
// shuffle feeding a `lane < k` block read inactive lanes).
template <class T> YM_INLINE T pin(T x) {
  asm volatile("" : "+v"(x));
  return x;
}
YM_INLINE uint32_t shfl(uint32_t x, int l) { return pin(__shfl(x, l, 64)); }
YM_INLINE uint64_t shfl(uint64_t x, int l) { return pin(__shfl(x, l, 64)); }
// inclusive sum over the wave in DPP (VALU lane moves, no LDS crossbar round trips): row_shr
// 1, 2, 4, 8 scans each row of 16 lanes, row_bcast:15 / row_bcast:31 carry the row totals
YM_INLINE uint32_t wincl(uint32_t x, uint32_t) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false); // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false); // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false); // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false); // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); // row_bcast:31 -> rows 2, 3
  return x;
}
// number of leading set bits of a lane mask (lanes 0.. that all satisfy a predicate)
YM_INLINE uint32_t lead_ones(uint64_t m) { return m == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~m); }

// ------------------------------------------------------------------ staged varints
// Branch-free LEB128 u32 at byte p of staged words (read_var_u32, yrs/src/encoding/varint.rs
// :244-260, wrapping_shl: a 5th byte contributes its low 4 bits): value, length; fine = it
// ends within 5 bytes and before `end`; canon = re-encoding gives the same bytes.
struct VarR {
  uint32_t v, n;
  bool fine, canon;
};
YM_INLINE VarR var_at(const uint32_t *w, uint32_t p, uint32_t end) {
  const uint32_t q = p >> 2;
  const uint64_t d = ((uint64_t)w[q + 1] << 32) | w[q];
  const uint64_t x = d >> ((p & 3) * 8); // >= 5 valid bytes
  const uint64_t stop = ~x & 0x8080808080ull;
  const uint32_t n = ((uint32_t)__builtin_ctzll(stop | (1ull << 47)) >> 3) + 1; // 6: no end in 5 bytes
  const uint32_t xl = (uint32_t)x;
  uint32_t v = (xl & 0x7Fu) | ((xl >> 1) & 0x3F80u) | ((xl >> 2) & 0x1FC000u) | ((xl >> 3) & 0xFE00000u) |
               ((uint32_t)(x >> 4) & 0xF0000000u);
  v &= n < 5 ? (1u << (7 * n)) - 1 : 0xFFFFFFFFu;
  const uint32_t last = (uint32_t)(x >> (8 * (n - 1))) & 0xFF;
  VarR r;
  r.v = v;
  r.n = n;
  r.fine = n <= 5 && p + n <= end;
  r.canon = n == 1 || (last != 0 && (n < 5 || last < 16));
  return r;
}

} // namespace ym
