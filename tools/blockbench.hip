// Diagnostic (not part of the engine): cycles of canon_size / emit_block (the fast path's sizes
// and write phases) per block of one document, on one lane.  Build: hipcc -O3 -std=c++17
// --offload-arch=gfx950 -I../y-crdt_amd/csrc blockbench.hip -o blockbench;
// run: ./blockbench doc.bin doc.off (u32 update offsets, n + 1 of them)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstring>
#include "ycodec.h"
#include "ykernels.h"
#include "ysm.h"
#include "ywin.h"
#include "yblock.h"

using namespace ym;

struct ListSink {
  uint32_t *bl; // 6 words per block: pos, client, clock, len, meta, ref
  uint32_t n, ubase;
  YM_INLINE void on_section(uint32_t) {}
  YM_INLINE int on_block(uint32_t client, uint32_t clock, const BlockInfo &bi, uint32_t bpos, uint32_t blen) {
    if (bi.kind == BK_SKIP) return 0;
    uint32_t *w = bl + 6 * n++;
    w[0] = ubase + bpos;
    w[1] = client;
    w[2] = clock;
    w[3] = bi.len;
    w[4] = (uint32_t)bi.kind | (bi.reenc ? 4u : 0u) | (bi.enc_panic ? 8u : 0u) | (blen << 8);
    w[5] = bi.ref;
    return 0;
  }
  YM_INLINE int on_ds_begin(uint32_t) { return 0; }
  YM_INLINE int on_ds_entry(uint32_t, uint32_t) { return 0; }
  YM_INLINE void on_ds_range(uint32_t, uint32_t) {}
  YM_INLINE int on_ds_done() { return 0; }
};

__global__ void __launch_bounds__(64) k_blocks(const uint8_t *doc, uint32_t nbytes, const uint32_t *uoff, uint32_t nu,
                                               uint32_t *bl, unsigned long long *out) {
  if (threadIdx.x) return;
  ym_set_grammar(0);
  ListSink s{bl, 0, 0};
  for (uint32_t u = 0; u < nu; u++) {
    WCur c;
    wc_init(c, doc + uoff[u], uoff[u + 1] - uoff[u]);
    s.ubase = uoff[u];
    smwalk_update(c, s);
  }
  out[0] = s.n;
  for (uint32_t k = 0; k < s.n; k++) {
    const uint32_t *w = bl + 6 * k;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const uint32_t sz = canon_size(doc, nbytes, w[0], w[1], w[2], w[3], w[4]);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[1 + 2 * k] = t1 - t0;
    out[2 + 2 * k] = sz;
  }
}

__global__ void __launch_bounds__(64) k_json(const uint8_t *js, uint32_t n, unsigned long long *out) {
  if (threadIdx.x) return;
  ym_set_grammar(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const bool pl = json_plain(js, n);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  Counter c;
  const int e = json_canon(js, n, c);
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
  out[0] = pl;
  out[1] = t1 - t0;
  out[2] = t2 - t1;
  out[3] = (unsigned long long)e;
  out[4] = c.n;
}

int main(int argc, char **argv) {
  if (argc > 3) { // json text timing
    const uint32_t n = (uint32_t)strlen(argv[3]);
    uint8_t *dj;
    unsigned long long *dout, o[5];
    hipMalloc(&dj, n + 64);
    hipMalloc(&dout, 64);
    hipMemcpy(dj, argv[3], n, hipMemcpyHostToDevice);
    for (int it = 0; it < 3; it++) {
      hipLaunchKernelGGL(k_json, dim3(1), dim3(64), 0, 0, dj, n, dout);
      hipMemcpy(o, dout, 40, hipMemcpyDeviceToHost);
      printf("json %u bytes: plain %llu (%llu cycles), json_canon %llu cycles err %llu size %llu\n", n, o[0], o[1],
             o[2], o[3], o[4]);
    }
  }
  FILE *fp = fopen(argv[1], "rb");
  std::vector<uint8_t> h(1 << 22);
  const size_t n = fread(h.data(), 1, h.size(), fp);
  fclose(fp);
  fp = fopen(argv[2], "rb");
  std::vector<uint32_t> off(1 << 16);
  const size_t no = fread(off.data(), 4, off.size(), fp);
  fclose(fp);
  uint8_t *dd;
  uint32_t *doff, *dbl;
  unsigned long long *dout;
  hipMalloc(&dd, n + 64);
  hipMalloc(&doff, no * 4);
  hipMalloc(&dbl, 6 * 4 * 65536);
  hipMalloc(&dout, 8 * (1 + 2 * 65536));
  hipMemcpy(dd, h.data(), n, hipMemcpyHostToDevice);
  hipMemcpy(doff, off.data(), no * 4, hipMemcpyHostToDevice);
  std::vector<unsigned long long> o(1 + 2 * 65536);
  std::vector<uint32_t> bl(6 * 65536);
  for (int it = 0; it < 2; it++) {
    hipLaunchKernelGGL(k_blocks, dim3(1), dim3(64), 0, 0, dd, (uint32_t)n, doff, (uint32_t)(no - 1), dbl, dout);
    hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost);
  }
  hipMemcpy(bl.data(), dbl, bl.size() * 4, hipMemcpyDeviceToHost);
  const uint32_t nb = (uint32_t)o[0];
  unsigned long long tot[16] = {0}, cnt[16] = {0}, mx[16] = {0};
  for (uint32_t k = 0; k < nb; k++) {
    const uint32_t ref = bl[6 * k + 5] & 15, reenc = (bl[6 * k + 4] & 4) != 0;
    const unsigned long long c = o[1 + 2 * k];
    tot[ref] += c;
    cnt[ref]++;
    if (c > mx[ref]) mx[ref] = c;
    (void)reenc;
  }
  printf("blocks %u\n", nb);
  for (int r = 0; r < 16; r++)
    if (cnt[r])
      printf("  ref %2d: %5llu blocks, canon_size cycles total %10llu mean %8llu max %8llu\n", r, cnt[r], tot[r],
             tot[r] / cnt[r], mx[r]);
  return 0;
}
