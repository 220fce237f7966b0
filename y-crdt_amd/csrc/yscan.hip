// yscan.hip — exclusive prefix sum over u64 (per-document sizes -> arena offsets).
// Three launches: per-tile totals, one-workgroup scan of the tile totals, per-tile
// rescan + add.  Tiles are 256 lanes x 8 elements, loads coalesced per lane group.
#include "ykernels.h"

namespace ym {
constexpr uint32_t SCAN_NT = 256, SCAN_IT = 8, SCAN_TILE = SCAN_NT * SCAN_IT;

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *sh, uint64_t &total) {
  uint32_t t = threadIdx.x, lane = t & 63, wid = t >> 6;
  uint64_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  if (t == 0) {
    uint64_t acc = 0;
    for (uint32_t w = 0; w < SCAN_NT / 64; w++) {
      uint64_t s = sh[w];
      sh[w] = acc;
      acc += s;
    }
    sh[SCAN_NT / 64] = acc;
  }
  __syncthreads();
  total = sh[SCAN_NT / 64];
  uint64_t r = sh[wid] + x - v;
  __syncthreads();
  return r;
}

// n_dev (optional): the element count is read on the device (<= the n the grid was sized
// for), so a scan can follow the kernel that produces its length without a host round trip
__device__ __forceinline__ uint32_t scan_n(uint32_t n, const uint32_t *n_dev) {
  const uint32_t m = n_dev ? *n_dev : n;
  return m < n ? m : n;
}
__global__ void __launch_bounds__(256) k_scan_tiles(const uint64_t *in, uint32_t n, uint64_t *tile_sum,
                                                   const uint32_t *n_dev) {
  __shared__ uint64_t sh[SCAN_NT / 64 + 1];
  n = scan_n(n, n_dev);
  if (blockIdx.x * SCAN_TILE >= n && blockIdx.x) return; // (uniform)
  uint32_t base = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_IT;
  uint64_t s = 0;
  for (uint32_t i = 0; i < SCAN_IT; i++)
    if (base + i < n) s += in[base + i];
  uint64_t tot;
  block_excl_scan(s, sh, tot);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(256) k_scan_top(uint64_t *tile_sum, uint32_t ntiles, uint32_t n,
                                                 const uint32_t *n_dev) {
  __shared__ uint64_t sh[SCAN_NT / 64 + 1];
  if (n_dev) {
    const uint32_t m = scan_n(n, n_dev);
    ntiles = m ? (m + SCAN_TILE - 1) / SCAN_TILE : 1;
  }
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < ntiles; b0 += SCAN_NT) {
    uint32_t i = b0 + threadIdx.x;
    uint64_t v = i < ntiles ? tile_sum[i] : 0, tot;
    uint64_t e = block_excl_scan(v, sh, tot);
    if (i < ntiles) tile_sum[i] = carry + e;
    carry += tot;
  }
  if (threadIdx.x == 0) tile_sum[ntiles] = carry;
}
__global__ void __launch_bounds__(256) k_scan_final(const uint64_t *in, uint32_t n, const uint64_t *tile_off,
                                                   uint64_t *out, const uint32_t *n_dev) {
  __shared__ uint64_t sh[SCAN_NT / 64 + 1];
  n = scan_n(n, n_dev);
  const uint32_t ntiles = n ? (n + SCAN_TILE - 1) / SCAN_TILE : 1;
  if (blockIdx.x >= ntiles) return; // (uniform)
  uint32_t base = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_IT;
  uint64_t v[SCAN_IT], s = 0;
  for (uint32_t i = 0; i < SCAN_IT; i++) {
    v[i] = base + i < n ? in[base + i] : 0;
    s += v[i];
  }
  uint64_t tot;
  uint64_t e = block_excl_scan(s, sh, tot) + tile_off[blockIdx.x];
  for (uint32_t i = 0; i < SCAN_IT; i++) {
    if (base + i < n) out[base + i] = e;
    e += v[i];
  }
  if (blockIdx.x == ntiles - 1 && threadIdx.x == 0) out[n] = tile_off[ntiles];
}

size_t scan_tmp_elems(uint32_t n) { return n / SCAN_TILE + 2; }
void launch_scan_u64(const uint64_t *in, uint64_t *out, uint32_t n, uint64_t *tmp, hipStream_t s,
                     const uint32_t *n_dev) {
  uint32_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (ntiles == 0) {
    hipMemsetAsync(out, 0, sizeof(uint64_t), s);
    return;
  }
  hipLaunchKernelGGL(k_scan_tiles, dim3(ntiles), dim3(SCAN_NT), 0, s, in, n, tmp, n_dev);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_NT), 0, s, tmp, ntiles, n, n_dev);
  hipLaunchKernelGGL(k_scan_final, dim3(ntiles), dim3(SCAN_NT), 0, s, in, n, tmp, out, n_dev);
}
} // namespace ym

namespace ym {
// pack per-document outputs (start, len) into a contiguous arena at pack_off[d]
// workgroup (x) per document; small batches also split each document over gridDim.y
// workgroups (one long document would otherwise be copied by one workgroup)
__global__ void __launch_bounds__(256) k_pack(const uint8_t *src, const uint64_t *start, const uint64_t *len,
                                             const uint64_t *pack_off, uint8_t *dst, uint32_t n_docs) {
  for (uint32_t d = blockIdx.x; d < n_docs; d += gridDim.x) {
    const uint8_t *s = src + start[d];
    uint8_t *o = dst + pack_off[d];
    const uint64_t n = len[d];
    const uint64_t part = (n + gridDim.y - 1) / gridDim.y, b0 = part * blockIdx.y;
    const uint64_t b1 = b0 + part < n ? b0 + part : n;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += 256) o[i] = s[i];
  }
}
void launch_pack(const uint8_t *src, const uint64_t *start, const uint64_t *len, const uint64_t *pack_off,
                 uint8_t *dst, uint32_t n_docs, hipStream_t s) {
  if (!n_docs) return;
  uint32_t g = n_docs < 8192 ? n_docs : 8192;
  const uint32_t ys = n_docs <= 64 ? 256 : n_docs <= 1024 ? 16 : 1;
  hipLaunchKernelGGL(k_pack, dim3(g, ys), dim3(256), 0, s, src, start, len, pack_off, dst, n_docs);
}

__global__ void __launch_bounds__(256) k_rebase_u64(uint64_t *a, uint64_t n, uint64_t sub) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) a[i] -= sub;
}
void launch_rebase_u64(uint64_t *a, uint64_t n, uint64_t sub, hipStream_t s) {
  if (!n || !sub) return;
  const uint64_t g = (n + 255) / 256;
  hipLaunchKernelGGL(k_rebase_u64, dim3(g < 4096 ? (uint32_t)g : 4096u), dim3(256), 0, s, a, n, sub);
}
} // namespace ym
