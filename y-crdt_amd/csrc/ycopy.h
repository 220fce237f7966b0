// ycopy.h — a workgroup copying one byte range together (long verbatim blocks: a pasted
// string of tens of KB copied by one lane held a trace document for milliseconds).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ym {
// n bytes src -> dst by the lanes t of nt: the head up to dst's 16-byte alignment and the tail
// byte by byte, the body as 16-byte stores of four dwords assembled from five aligned source
// dwords (v_alignbyte).  Reads up to 4 bytes past src + n (the arenas carry 16 readable bytes).
__device__ __forceinline__ void copy_coop(uint8_t *dst, const uint8_t *src, uint32_t n, uint32_t t, uint32_t nt) {
  const uint32_t head0 = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15), h = head0 < n ? head0 : n;
  if (t < h) dst[t] = src[t];
  const uint32_t body = (n - h) & ~15u;
  const uint8_t *s = src + h;
  uint8_t *d = dst + h;
  const uint32_t sh = (uint32_t)((uintptr_t)s & 3);
  const uint32_t *sw = (const uint32_t *)((uintptr_t)s - sh);
  for (uint32_t o = 16 * t; o < body; o += 16 * nt) {
    const uint32_t *p = sw + o / 4;
    const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = sh ? p[4] : 0u;
    uint4 v;
    v.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
    v.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
    v.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
    v.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
    *(uint4 *)(d + o) = v;
  }
  for (uint32_t q = h + body + t; q < n; q += nt) dst[q] = src[q];
}
} // namespace ym
