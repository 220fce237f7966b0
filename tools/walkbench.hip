// Diagnostic (not part of the engine): cycles of one exact state-machine walk (ysm.h) of one
// update staged in LDS, as k_decode_exact walks it (one wavefront in lockstep), with a
// per-state cycle histogram.  Build: hipcc -O3 -std=c++17 --offload-arch=gfx950
// -I../y-crdt_amd/csrc walkbench.hip -o walkbench; run: ./walkbench update.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__shared__ unsigned long long wb_t;
__shared__ unsigned wb_prev;
__shared__ unsigned long long wb_hist[32];
__shared__ unsigned wb_cnt[32];
#define YM_SM_PROBE(st)                                        \
  do {                                                         \
    const unsigned long long _n = __builtin_amdgcn_s_memtime(); \
    if (threadIdx.x == 0) {                                    \
      wb_hist[wb_prev] += _n - wb_t;                           \
      wb_cnt[wb_prev]++;                                       \
      wb_prev = (st);                                          \
      wb_t = _n;                                               \
    }                                                          \
  } while (0)
#include "ycodec.h"
#include "ykernels.h"
#include "ysm.h"
#include "ylds.h"
#include "yblock.h"

using namespace ym;

template <bool PROBE>
__global__ void __launch_bounds__(256) k_walk(const uint8_t *u, uint32_t len, uint32_t *ovf, unsigned long long *out) {
  __shared__ __align__(16) uint32_t stage[DEC_STAGE / 4 + 4];
  for (uint32_t q = threadIdx.x; q < (len + 3) / 4; q += blockDim.x) {
    uint32_t w = 0;
    for (uint32_t k = 0; k < 4; k++)
      if (4 * q + k < len) w |= (uint32_t)u[4 * q + k] << (8 * k);
    stage[q] = w;
  }
  if (threadIdx.x < 32) {
    wb_hist[threadIdx.x] = 0;
    wb_cnt[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) wb_prev = 31;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  ym_set_grammar(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  RegSink s;
  s.nb = s.ne = s.nr = 0;
  s.unsupported = s.big_ds = false;
  s.ubase = 0;
  SCurU c;
  c.p = (const uint8_t *)stage;
  c.n = len;
  c.i = 0;
  c.w = stage;
  c.base = 0;
  const int e = smwalk_update(c, s);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  OvfFill f{ovf, s.nb, s.ne, 0, 0, 0};
  f.on = threadIdx.x == 0;
  SCurU c2;
  c2.p = (const uint8_t *)stage;
  c2.n = len;
  c2.i = 0;
  c2.w = stage;
  c2.base = 0;
  smwalk_update(c2, f);
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = (unsigned long long)e;
    out[1] = t1 - t0;
    out[2] = t2 - t1;
    out[3] = s.nb;
    out[4] = s.ne;
    out[5] = s.nr;
    for (int k = 0; k < 32; k++) {
      out[8 + k] = wb_hist[k];
      out[40 + k] = wb_cnt[k];
    }
  }
}

int main(int argc, char **argv) {
  FILE *fp = fopen(argv[1], "rb");
  std::vector<uint8_t> h(1 << 16);
  const size_t n = fread(h.data(), 1, h.size(), fp);
  fclose(fp);
  uint8_t *du;
  uint32_t *dov;
  unsigned long long *dout;
  hipMalloc(&du, n + 64);
  hipMalloc(&dov, 1 << 20);
  hipMalloc(&dout, 128 * 8);
  hipMemcpy(du, h.data(), n, hipMemcpyHostToDevice);
  std::vector<unsigned long long> o(128);
  static const char *names[] = {"NCL", "NB", "CLIENT", "CLOCK", "INFO", "GCLEN", "OC", "OK", "RC", "RK", "PI",
                                "PNAME", "PC", "PK", "PSUB", "CDEL", "CSTR", "NDS", "DCL", "DNR", "DST", "DLN"};
  for (int it = 0; it < 3; it++) {
    hipLaunchKernelGGL(k_walk<true>, dim3(1), dim3(256), 0, 0, du, (uint32_t)n, dov, dout);
    hipMemcpy(o.data(), dout, 128 * 8, hipMemcpyDeviceToHost);
    printf("bytes %zu err %llu walk %llu cycles, ovf walk %llu cycles, blocks %llu entries %llu ranges %llu\n", n, o[0],
           o[1], o[2], o[3], o[4], o[5]);
  }
  for (int k = 0; k < 22; k++)
    if (o[40 + k]) printf("  %-7s steps %6llu cycles %10llu (%.0f per step)\n", names[k], o[40 + k], o[8 + k],
                          (double)o[8 + k] / o[40 + k]);
  return 0;
}
