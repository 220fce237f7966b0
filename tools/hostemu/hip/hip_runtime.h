// Host emulation of the few HIP names used by the lane-per-document device code
// (ycompact.hip and the headers it includes), so that the same source runs on the CPU in the
// parity tests (tests/test_compact_emu.py).  Test tooling: never linked into the product.
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>
#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __align__(n) alignas(n)
#define __shared__
#define __constant__
#define __launch_bounds__(...)
typedef void *hipStream_t;
struct dim3 {
  unsigned x, y, z;
  dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct uint4 {
  uint32_t x, y, z, w;
};
struct emu_idx {
  unsigned x, y, z;
};
static emu_idx blockIdx, threadIdx;
#define hipLaunchKernelGGL(...) ((void)0)
#define __builtin_amdgcn_s_memtime() 0ull
static inline int __clz(int x) { return x ? __builtin_clz((unsigned)x) : 32; }
static inline int __clzll(long long x) { return x ? __builtin_clzll((unsigned long long)x) : 64; }
static inline long long __double_as_longlong(double d) {
  long long v;
  memcpy(&v, &d, 8);
  return v;
}
