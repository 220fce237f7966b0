// ymerge_host.cpp — host engine behind include/ymerge.h.
//
// Owns one HIP stream + HBM workspace per context and sequences the gfx950
// kernels of a batch:
//   count/validate -> scratch offsets (scan) -> plan (sizes) -> out offsets (scan)
//   -> write.
// The product path is the HIP path only: if no device is usable every call fails
// with YMERGE_ERR_DEVICE (there is no CPU fallback).
#include "../../include/ymerge.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "ykernels.h"

namespace {

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap && p) return true;
    size_t want = std::max(bytes, cap + cap / 2);
    if (want < 256) want = 256;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, want) != hipSuccess) return false;
    cap = want;
    return true;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T *as() const { return (T *)p; }
};

thread_local uint8_t g_last_error = 0;

} // namespace

struct ymerge_ctx {
  int device = 0;
  hipStream_t s = nullptr;
  DevBuf in_bytes, in_upd_off, in_doc_upd, in_sv, in_sv_off;
  DevBuf status, counts, need, scr_off, scratch, sizes, out_off, out, scan_tmp;
  uint64_t *h_pinned = nullptr;
  hipEvent_t ev[6];
  ymerge_stats stats{};
  std::mutex mu;
};

static bool ctx_init(ymerge_ctx *c, int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device >= n || device < 0) return false;
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) return false;
  if (hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess) return false;
  if (hipHostMalloc((void **)&c->h_pinned, 64 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess) return false;
  for (auto &e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) return false;
  return true;
}

extern "C" ymerge_ctx *ymerge_ctx_create(int device) {
  auto *c = new ymerge_ctx();
  if (!ctx_init(c, device)) {
    delete c;
    return nullptr;
  }
  return c;
}

extern "C" void ymerge_ctx_destroy(ymerge_ctx *c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->s) hipStreamSynchronize(c->s);
  for (DevBuf *b : {&c->in_bytes, &c->in_upd_off, &c->in_doc_upd, &c->in_sv, &c->in_sv_off, &c->status, &c->counts,
                    &c->need, &c->scr_off, &c->scratch, &c->sizes, &c->out_off, &c->out, &c->scan_tmp})
    b->release();
  if (c->h_pinned) hipHostFree(c->h_pinned);
  for (auto &e : c->ev)
    if (e) hipEventDestroy(e);
  if (c->s) hipStreamDestroy(c->s);
  delete c;
}

static bool read_u64(ymerge_ctx *c, const uint64_t *d_src, uint64_t &v) {
  if (hipMemcpyAsync(c->h_pinned, d_src, sizeof(uint64_t), hipMemcpyDeviceToHost, c->s) != hipSuccess) return false;
  if (hipStreamSynchronize(c->s) != hipSuccess) return false;
  v = c->h_pinned[0];
  return true;
}

static int merge_device(ymerge_ctx *c, const uint8_t *d_bytes, const uint64_t *d_upd_off, const uint64_t *d_doc_upd,
                        uint64_t n_docs, ymerge_device_result *res) {
  if (hipSetDevice(c->device) != hipSuccess) return YMERGE_ERR_DEVICE;
  if (n_docs > 0xFFFFFFFFull) return YMERGE_ERR_OTHER;
  uint32_t n = (uint32_t)n_docs;
  ym::BatchIn b{d_bytes, d_upd_off, d_doc_upd, n};
  size_t nn = (size_t)n + 1;
  if (!c->status.ensure(nn) || !c->counts.ensure(4 * nn * 4) || !c->need.ensure(nn * 8) ||
      !c->scr_off.ensure(nn * 8) || !c->sizes.ensure(nn * 8) || !c->out_off.ensure(nn * 8) ||
      !c->scan_tmp.ensure(ym::scan_tmp_elems(n) * 8 + 64))
    return YMERGE_ERR_DEVICE;
  hipEventRecord(c->ev[0], c->s);
  ym::launch_seq_count(b, c->status.as<uint8_t>(), c->counts.as<uint32_t>(), c->need.as<uint64_t>(), c->s);
  ym::launch_scan_u64(c->need.as<uint64_t>(), c->scr_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
  hipEventRecord(c->ev[1], c->s);
  uint64_t words = 0;
  if (!read_u64(c, c->scr_off.as<uint64_t>() + n, words)) return YMERGE_ERR_DEVICE;
  if (!c->scratch.ensure((size_t)words * 4 + 64)) return YMERGE_ERR_DEVICE;
  hipEventRecord(c->ev[2], c->s);
  ym::launch_seq_merge(false, b, c->status.as<uint8_t>(), c->counts.as<uint32_t>(), c->scr_off.as<uint64_t>(),
                       c->scratch.as<uint32_t>(), c->sizes.as<uint64_t>(), nullptr, nullptr, c->status.as<uint8_t>(),
                       c->s);
  ym::launch_scan_u64(c->sizes.as<uint64_t>(), c->out_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
  hipEventRecord(c->ev[3], c->s);
  uint64_t total = 0;
  if (!read_u64(c, c->out_off.as<uint64_t>() + n, total)) return YMERGE_ERR_DEVICE;
  if (!c->out.ensure((size_t)total + 64)) return YMERGE_ERR_DEVICE;
  hipEventRecord(c->ev[4], c->s);
  ym::launch_seq_merge(true, b, c->status.as<uint8_t>(), c->counts.as<uint32_t>(), c->scr_off.as<uint64_t>(),
                       c->scratch.as<uint32_t>(), nullptr, c->out_off.as<uint64_t>(), c->out.as<uint8_t>(), nullptr,
                       c->s);
  hipEventRecord(c->ev[5], c->s);
  if (hipStreamSynchronize(c->s) != hipSuccess) return YMERGE_ERR_DEVICE;
  if (hipGetLastError() != hipSuccess) return YMERGE_ERR_DEVICE;
  float t01 = 0, t23 = 0, t45 = 0, t05 = 0;
  hipEventElapsedTime(&t01, c->ev[0], c->ev[1]);
  hipEventElapsedTime(&t23, c->ev[2], c->ev[3]);
  hipEventElapsedTime(&t45, c->ev[4], c->ev[5]);
  hipEventElapsedTime(&t05, c->ev[0], c->ev[5]);
  c->stats = ymerge_stats{};
  c->stats.n_docs = n_docs;
  c->stats.bytes_out = total;
  c->stats.docs_exact = n_docs;
  c->stats.ms_count = t01;
  c->stats.ms_plan = t23;
  c->stats.ms_write = t45;
  c->stats.ms_total = t05;
  res->d_out = c->out.as<uint8_t>();
  res->d_out_off = c->out_off.as<uint64_t>();
  res->d_status = c->status.as<uint8_t>();
  res->out_bytes = total;
  return 0;
}

extern "C" int ymerge_updates_v1_batch_device(ymerge_ctx *c, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                                              const uint64_t *d_doc_upd, uint64_t n_docs, ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return merge_device(c, d_bytes, d_upd_off, d_doc_upd, n_docs, res);
}

extern "C" int yencode_state_vector_from_update_v1_batch_device(ymerge_ctx *, const uint8_t *, const uint64_t *,
                                                                uint64_t, ymerge_device_result *) {
  return YMERGE_ERR_UNSUPPORTED;
}
extern "C" int ydiff_updates_v1_batch_device(ymerge_ctx *, const uint8_t *, const uint64_t *, const uint8_t *,
                                             const uint64_t *, uint64_t, ymerge_device_result *) {
  return YMERGE_ERR_UNSUPPORTED;
}

extern "C" int ymerge_result_to_host(ymerge_ctx *c, const ymerge_device_result *res, uint64_t n_docs, uint8_t *out,
                                     uint64_t *out_off, uint8_t *status) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  if (out && res->out_bytes &&
      hipMemcpyAsync(out, res->d_out, res->out_bytes, hipMemcpyDeviceToHost, c->s) != hipSuccess)
    return YMERGE_ERR_DEVICE;
  if (out_off &&
      hipMemcpyAsync(out_off, res->d_out_off, (n_docs + 1) * 8, hipMemcpyDeviceToHost, c->s) != hipSuccess)
    return YMERGE_ERR_DEVICE;
  if (status && n_docs && hipMemcpyAsync(status, res->d_status, n_docs, hipMemcpyDeviceToHost, c->s) != hipSuccess)
    return YMERGE_ERR_DEVICE;
  return hipStreamSynchronize(c->s) == hipSuccess ? 0 : YMERGE_ERR_DEVICE;
}

extern "C" void ymerge_last_stats(ymerge_ctx *c, ymerge_stats *st) {
  if (c && st) *st = c->stats;
}

extern "C" int ymerge_updates_v1_batch(ymerge_ctx *c, const uint8_t *bytes, const uint64_t *upd_off,
                                       uint64_t n_updates, const uint64_t *doc_upd, uint64_t n_docs,
                                       ymerge_batch_result **out) {
  if (!c || !out) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  uint64_t nbytes = upd_off[n_updates];
  if (!c->in_bytes.ensure(nbytes + 16) || !c->in_upd_off.ensure((n_updates + 1) * 8) ||
      !c->in_doc_upd.ensure((n_docs + 1) * 8))
    return YMERGE_ERR_DEVICE;
  if (nbytes && hipMemcpyAsync(c->in_bytes.p, bytes, nbytes, hipMemcpyHostToDevice, c->s) != hipSuccess)
    return YMERGE_ERR_DEVICE;
  if (hipMemcpyAsync(c->in_upd_off.p, upd_off, (n_updates + 1) * 8, hipMemcpyHostToDevice, c->s) != hipSuccess ||
      hipMemcpyAsync(c->in_doc_upd.p, doc_upd, (n_docs + 1) * 8, hipMemcpyHostToDevice, c->s) != hipSuccess)
    return YMERGE_ERR_DEVICE;
  ymerge_device_result dr{};
  int st = merge_device(c, c->in_bytes.as<uint8_t>(), c->in_upd_off.as<uint64_t>(), c->in_doc_upd.as<uint64_t>(),
                        n_docs, &dr);
  if (st) return st;
  auto *r = (ymerge_batch_result *)calloc(1, sizeof(ymerge_batch_result));
  r->n_docs = n_docs;
  r->out_bytes = dr.out_bytes;
  r->out = (uint8_t *)malloc(dr.out_bytes + 1);
  r->out_off = (uint64_t *)malloc((n_docs + 1) * 8);
  r->status = (uint8_t *)malloc(n_docs + 1);
  hipMemcpyAsync(r->out, dr.d_out, dr.out_bytes, hipMemcpyDeviceToHost, c->s);
  hipMemcpyAsync(r->out_off, dr.d_out_off, (n_docs + 1) * 8, hipMemcpyDeviceToHost, c->s);
  hipMemcpyAsync(r->status, dr.d_status, n_docs, hipMemcpyDeviceToHost, c->s);
  if (hipStreamSynchronize(c->s) != hipSuccess) {
    ymerge_batch_result_destroy(r);
    return YMERGE_ERR_DEVICE;
  }
  *out = r;
  return 0;
}

extern "C" void ymerge_batch_result_destroy(ymerge_batch_result *r) {
  if (!r) return;
  free(r->out);
  free(r->out_off);
  free(r->status);
  free(r);
}

// ---------------------------------------------------------------- single document API
static std::mutex g_default_mu;
static ymerge_ctx *g_default = nullptr;
static ymerge_ctx *default_ctx() {
  std::lock_guard<std::mutex> g(g_default_mu);
  if (!g_default) g_default = ymerge_ctx_create(0);
  return g_default;
}

extern "C" uint8_t ymerge_last_error(void) { return g_last_error; }

extern "C" char *ymerge_updates_v1(const char *const *updates, const uint32_t *updates_len, uint32_t updates_count,
                                   uint32_t *out_len) {
  g_last_error = 0;
  ymerge_ctx *c = default_ctx();
  if (!c) {
    g_last_error = YMERGE_ERR_DEVICE;
    return nullptr;
  }
  std::vector<uint64_t> off(updates_count + 1);
  uint64_t tot = 0;
  for (uint32_t i = 0; i < updates_count; i++) {
    off[i] = tot;
    tot += updates_len[i];
  }
  off[updates_count] = tot;
  std::vector<uint8_t> arena(tot + 1);
  for (uint32_t i = 0; i < updates_count; i++)
    if (updates_len[i]) memcpy(arena.data() + off[i], updates[i], updates_len[i]);
  uint64_t doc_upd[2] = {0, updates_count};
  ymerge_batch_result *r = nullptr;
  int st = ymerge_updates_v1_batch(c, arena.data(), off.data(), updates_count, doc_upd, 1, &r);
  if (st) {
    g_last_error = (uint8_t)st;
    return nullptr;
  }
  if (r->status[0]) {
    g_last_error = r->status[0];
    ymerge_batch_result_destroy(r);
    return nullptr;
  }
  uint64_t n = r->out_off[1] - r->out_off[0];
  char *res = (char *)malloc(n ? n : 1);
  memcpy(res, r->out + r->out_off[0], n);
  *out_len = (uint32_t)n;
  ymerge_batch_result_destroy(r);
  return res;
}

extern "C" char *ydiff_updates_v1(const char *, uint32_t, const char *, uint32_t, uint32_t *) {
  g_last_error = YMERGE_ERR_UNSUPPORTED;
  return nullptr;
}
extern "C" char *yencode_state_vector_from_update_v1(const char *, uint32_t, uint32_t *) {
  g_last_error = YMERGE_ERR_UNSUPPORTED;
  return nullptr;
}

extern "C" void ybinary_destroy(char *ptr, uint32_t) { free(ptr); }
