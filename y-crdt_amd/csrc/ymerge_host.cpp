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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
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
// Provenance of the last YMERGE_ERR_DEVICE on this thread: the failing stage (file:line or a
// name) and the HIP error, kept until the next device failure (ymerge_last_error_message);
// also printed to stderr when env YMERGE_VERBOSE is set.
thread_local char g_last_msg[256] = "";
int dev_err(const char *where, hipError_t e = hipSuccess) {
  static const bool verbose = getenv("YMERGE_VERBOSE") != nullptr;
  if (e == hipSuccess) e = hipPeekAtLastError();
  snprintf(g_last_msg, sizeof g_last_msg, "device error at %s: %s (%d)", where,
           e == hipSuccess ? "allocation or bound" : hipGetErrorString(e), (int)e);
  if (verbose) fprintf(stderr, "ymerge: %s\n", g_last_msg);
  return YMERGE_ERR_DEVICE;
}
#define YM_STR2(x) #x
#define YM_STR(x) YM_STR2(x)
#define DEV_FAIL() dev_err("ymerge_host.cpp:" YM_STR(__LINE__))
ymerge_batch_result *alloc_result(uint64_t n_docs, uint64_t out_bytes);

} // namespace

struct ymerge_ctx {
  int device = 0;
  hipStream_t s = nullptr;
  DevBuf in_bytes, in_upd_off, in_doc_upd, in_sv, in_sv_off, sync_off, sync_end, sync_st;
  DevBuf status, path, out_start, out_len, pack_off, counts, need, scr_off, scratch, sizes, spill_off, scan_tmp;
  DevBuf arena, packed, counter, stamps, plan_small, plan_big, rec, ovf, big_scratch, lean_scr, lean_tot, cscr;
  DevBuf gs_list, gs1, gs2; // long single-client documents (ygiant.hip)
  DevBuf big_list;          // documents handed to the tiled kernel (k_fast_merge), its launch list
  DevBuf huge;              // k_decode's list of long updates, overflow bump counter
  DevBuf lp;                // the parallel parse of long updates (ylong.hip): scratch
  bool long_parse = true;   // env YMERGE_LONG_PARSE=0: every long update takes the exact walk
  bool tiny_forced = false; // env YMERGE_TINY set
  uint32_t seq_lpw = 0; // env YMERGE_SEQ_LPW: exact-engine documents per wavefront (0: by count)
  uint32_t lp_mid = ym::LP_MID_LEN; // env YMERGE_LP_MID: staged rich updates of >= this many bytes -> parallel parse
  bool long_grid = true;    // env YMERGE_LONG_GRID=0: single long update documents take the tiled kernel / planners
  uint32_t ls_min_diff = ym::LS_MIN_DIFF; // diff / SV documents on the long-update grid path (env YMERGE_LS_MIN)
  DevBuf ls_list, ls_scr, ls_done, ls_ovf; // their list, per-document scratch, planner skip flags, records
  DevBuf lean_ord;          // k_lean dispatch order: 8 counters, then n_docs document indices
  DevBuf plan_wlist;        // diff / SV: documents k_plan_lane leaves to k_plan_wave
  DevBuf lean_dbg;          // YMERGE_LEAN_DEBUG hand-over reasons (this context's device only)
  uint64_t lean_scr_max = ~0ull; // env YMERGE_LEAN_SCR_MAX: cap on the k_lean BIG-mode scratch (tests)
  // lib0 v2: v1x arena + offsets + per-update status, v2 output arena + sizes + offsets,
  // state-vector rest offsets + pre-status
  DevBuf v2x, v2x_sz, v2x_off, v2_ust, v2_out, v2_osz, v2_ooff, v2_svoff, v2_svend, v2_pre;
  DevBuf v2_scr, v2_colsz, v2_over; // one-pass EncoderV2: column streams, sizes, overflow flag
  bool v2_onepass = true;           // env YMERGE_V2_ONEPASS=0: counting walk + writing walk
  bool want_stamps = false;
  uint64_t *h_pinned = nullptr;
  // k_lean's result words (hand-overs, output bytes) written by k_lean_fin into host-mapped
  // memory behind a sequence number the host polls: no D2H copy, no stream-sync wake-up
  // (env YMERGE_LEAN_SPIN=0: copy + hipStreamSynchronize)
  uint32_t *h_sig = nullptr, *d_sig = nullptr;
  // the one-long-document lane (C1) replayed as a captured hipGraph: its ~35 small launches
  // are host-bound at several us each.  A key (inputs + buffer addresses) seen twice in a row
  // is captured on its second run and replayed after (env YMERGE_GIANT_GRAPH=0: eager).
  uint64_t giant_key = 0, graph_key = 0;
  hipGraphExec_t giant_exec = nullptr;
  bool giant_graph = true;
  uint32_t sig_seq = 0;
  bool lean_spin = true;
  bool timing = true; // stage timing events (ymerge_ctx_set_stage_timing)
  void *counters_clean = nullptr; // k_lean_fin left `counter` zeroed (this allocation): no memset
  hipEvent_t ev[10];
  hipEvent_t v2ev[4] = {}; // lib0 v2 merge: start, after the v2 -> v1x transcode, after the merge, after the encode
  ymerge_stats stats{};
  uint64_t stamps_docs = 0; // documents covered by `stamps` (last merge batch)
  // tiny-document updates / bytes, blocks (must equal FAST_BCAP, ymerge_fast.hip), DS entries, DS ranges
  ym::FastCaps caps{4, 4096, 1024, 512, 512};
  int fast_threads = 256;
  bool lean = true; // k_lean first (env YMERGE_LEAN=0: every document through k_decode + k_fast_merge)
  bool pack_stale = false; // pack_off not computed for the last merge (all documents on k_lean)
  bool times_pending = false; // the last merge's stage times wait on its events (resolve_times)
  uint32_t giant_min = ym::GS_MIN_U; // updates of a document for the grid-wide path (env YMERGE_GIANT_MIN, 0: off)
  bool giant_lane = true; // a batch of one such document skips the per-document routing (env YMERGE_GIANT_LANE=0: off)
  int lean_order = -1; // k_lean longest-first dispatch: env YMERGE_LEAN_ORDER 0/1, default for >= 8192 small docs
  // diff / SV common-shape planner (env YMERGE_PLANNER): 0 "lane" k_plan_lane + k_plan_wave for
  // long updates (default: C5 k_plan 4.24 -> 3.3 ms against the ring planner), 1 "ring"
  // k_plan_ring, 2 "wave" k_plan_wave for every document
  uint32_t planner = 0;
  uint32_t compact_lpw = 16; // k_compact documents per wavefront (env YMERGE_COMPACT_LPW; C2: 16 best)
  // host staging: two pinned buffers (double-buffered H2D / D2H of caller memory)
  uint8_t *stage[2] = {nullptr, nullptr};
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  // pipelined host merge: input / output copy streams, per-group events, packed ping-pong
  hipStream_t s_in = nullptr, s_out = nullptr;
  hipEvent_t ev_in[64] = {}, ev_out[2] = {}, ev_packed[2] = {};
  DevBuf packed2[2], grp_doc_upd;
  std::mutex mu;
};

static bool ctx_init(ymerge_ctx *c, int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device >= n || device < 0) return false;
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) return false;
  if (hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess) return false;
  if (hipHostMalloc((void **)&c->h_pinned, 1024 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess) return false;
  for (auto &e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) return false;
  for (auto &e : c->v2ev)
    if (hipEventCreate(&e) != hipSuccess) return false;
  // YMERGE_FAST_THREADS: workgroup size of the fast path (256/512/1024); 0 routes every
  // document through the exact engine (used by the parity tests to cover both engines)
  if (const char *v = getenv("YMERGE_FAST_THREADS")) c->fast_threads = atoi(v);
  if (const char *v = getenv("YMERGE_STAMPS")) c->want_stamps = atoi(v) != 0;
  if (const char *v = getenv("YMERGE_TINY")) { // 0: no tiny path; set: used at any batch size
    c->caps.in_cap = (uint32_t)atoi(v);
    c->tiny_forced = true;
  }
  if (const char *v = getenv("YMERGE_LEAN")) c->lean = atoi(v) != 0;
  if (const char *v = getenv("YMERGE_COMPACT_LPW")) c->compact_lpw = (uint32_t)atoi(v);
  if (const char *v = getenv("YMERGE_GIANT_MIN")) c->giant_min = (uint32_t)atoi(v);
  if (const char *v = getenv("YMERGE_GIANT_LANE")) c->giant_lane = atoi(v) != 0;
  if (const char *v = getenv("YMERGE_LEAN_ORDER")) c->lean_order = atoi(v);
  if (const char *v = getenv("YMERGE_LEAN_SPIN")) c->lean_spin = atoi(v) != 0;
  if (const char *v = getenv("YMERGE_V2_ONEPASS")) c->v2_onepass = atoi(v) != 0;
  if (const char *v = getenv("YMERGE_GIANT_GRAPH")) c->giant_graph = atoi(v) != 0;
  if (const char *v = getenv("YMERGE_PLANNER"))
    c->planner = strcmp(v, "ring") == 0 ? 1u : strcmp(v, "wave") == 0 ? 2u : 0u;
  if (const char *v = getenv("YMERGE_LEAN_SCR_MAX")) c->lean_scr_max = strtoull(v, nullptr, 10);
  if (const char *v = getenv("YMERGE_LONG_PARSE")) c->long_parse = atoi(v) != 0;
  if (const char *v = getenv("YMERGE_IDENTITY")) c->caps.ident = atoi(v) != 0;
  if (const char *v = getenv("YMERGE_SEQ_LPW")) c->seq_lpw = (uint32_t)std::min(64, std::max(0, atoi(v)));
  if (const char *v = getenv("YMERGE_LP_MID")) c->lp_mid = (uint32_t)std::max(1, atoi(v));
  if (const char *v = getenv("YMERGE_LONG_GRID")) c->long_grid = atoi(v) != 0;
  if (const char *v = getenv("YMERGE_LS_MIN")) c->ls_min_diff = (uint32_t)atoi(v);
  // the fast kernel's LDS layout must fit one workgroup (160 KB on gfx950)
  int lds_max = 0;
  if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess) return false;
  if (ym::fast_lds_bytes(c->caps) > (size_t)lds_max) {
    fprintf(stderr, "ymerge: fast-path LDS layout %zu B exceeds %d B\n", ym::fast_lds_bytes(c->caps), lds_max);
    return false;
  }
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
  for (DevBuf *b : {&c->in_bytes, &c->in_upd_off, &c->in_doc_upd, &c->in_sv, &c->in_sv_off, &c->sync_off,
                    &c->sync_end, &c->sync_st, &c->rec, &c->ovf, &c->status, &c->path,
                    &c->out_start, &c->out_len, &c->pack_off, &c->counts, &c->need, &c->scr_off, &c->scratch,
                    &c->sizes, &c->spill_off, &c->scan_tmp, &c->arena, &c->packed, &c->counter, &c->stamps,
                    &c->plan_small, &c->plan_big, &c->big_scratch, &c->lean_scr, &c->lean_tot, &c->cscr, &c->gs_list, &c->gs1, &c->gs2, &c->big_list, &c->huge, &c->lp, &c->ls_list, &c->ls_scr, &c->ls_done, &c->ls_ovf, &c->lean_ord, &c->lean_dbg, &c->plan_wlist, &c->v2x, &c->v2x_sz, &c->v2x_off, &c->v2_ust,
                    &c->v2_out, &c->v2_osz, &c->v2_ooff, &c->v2_svoff, &c->v2_svend, &c->v2_pre, &c->v2_scr,
                    &c->v2_colsz, &c->v2_over})
    b->release();
  if (c->h_pinned) hipHostFree(c->h_pinned);
  if (c->h_sig) hipHostFree(c->h_sig);
  if (c->giant_exec) hipGraphExecDestroy(c->giant_exec);
  for (int k = 0; k < 2; k++) {
    if (c->stage[k]) hipHostFree(c->stage[k]);
    if (c->stage_ev[k]) hipEventDestroy(c->stage_ev[k]);
    if (c->ev_out[k]) hipEventDestroy(c->ev_out[k]);
    if (c->ev_packed[k]) hipEventDestroy(c->ev_packed[k]);
    c->packed2[k].release();
  }
  for (auto &e : c->ev_in)
    if (e) hipEventDestroy(e);
  c->grp_doc_upd.release();
  if (c->s_in) hipStreamDestroy(c->s_in);
  if (c->s_out) hipStreamDestroy(c->s_out);
  for (auto &e : c->ev)
    if (e) hipEventDestroy(e);
  for (auto &e : c->v2ev)
    if (e) hipEventDestroy(e);
  if (c->s) hipStreamDestroy(c->s);
  delete c;
}

static bool read_words(ymerge_ctx *c, const void *d_src, size_t bytes, uint64_t *dst) {
  if (hipMemcpyAsync(c->h_pinned, d_src, bytes, hipMemcpyDeviceToHost, c->s) != hipSuccess) return false;
  if (hipStreamSynchronize(c->s) != hipSuccess) return false;
  memcpy(dst, c->h_pinned, bytes);
  return true;
}

// ---------------------------------------------------------------- host staging
// Caller memory is usually pageable: the HIP runtime then copies through its own small
// bounce buffers at a fraction of PCIe.  Large transfers go through two pinned 32 MB
// buffers instead: the host threads copy chunk k + 1 while the DMA engine moves chunk k.
constexpr size_t STAGE_CHUNK = 32u << 20;
static unsigned stage_threads() { // env YMERGE_STAGE_THREADS
  static const unsigned t = [] {
    if (const char *v = getenv("YMERGE_STAGE_THREADS")) return (unsigned)std::max(1, atoi(v));
    const unsigned h = std::thread::hardware_concurrency();
    return h >= 16 ? 8u : (h >= 4 ? h / 2 : 1u);
  }();
  return t;
}
// Persistent copy threads: a 265 MB host entry is ~10 large copies, and starting seven
// threads per copy cost more than the copies' tail (worker i takes slice i, the caller
// slice 0; one user at a time, a second concurrent user starts its own threads)
struct CopyPool {
  std::mutex use, m;
  std::condition_variable cv, done;
  uint64_t gen = 0;
  unsigned pending = 0, t = 0;
  uint8_t *dst = nullptr;
  const uint8_t *src = nullptr;
  size_t n = 0, per = 0;
  explicit CopyPool(unsigned threads) : t(threads) {
    for (unsigned i = 1; i < t; i++) std::thread([this, i] { worker(i); }).detach();
  }
  void worker(unsigned i) {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(m);
      cv.wait(lk, [&] { return gen != seen; });
      seen = gen;
      uint8_t *d = dst;
      const uint8_t *s = src;
      const size_t a = i * per, len = a < n ? std::min(per, n - a) : 0;
      lk.unlock();
      if (len) memcpy(d + a, s + a, len);
      lk.lock();
      if (--pending == 0) done.notify_one();
    }
  }
  void copy(void *d, const void *s, size_t bytes) {
    {
      std::lock_guard<std::mutex> lk(m);
      dst = (uint8_t *)d;
      src = (const uint8_t *)s;
      n = bytes;
      per = (bytes + t - 1) / t;
      pending = t - 1;
      gen++;
    }
    cv.notify_all();
    memcpy(d, s, std::min(per, bytes));
    std::unique_lock<std::mutex> lk(m);
    done.wait(lk, [&] { return pending == 0; });
  }
};
static void par_memcpy(void *dst, const void *src, size_t n) {
  const unsigned t = n >= (4u << 20) ? stage_threads() : 1;
  if (t <= 1) {
    memcpy(dst, src, n);
    return;
  }
  static CopyPool *pool = new CopyPool(t); // (never destroyed: detached workers outlive it otherwise)
  if (pool->use.try_lock()) {
    pool->copy(dst, src, n);
    pool->use.unlock();
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (n + t - 1) / t;
  for (unsigned i = 1; i < t; i++) {
    const size_t a = i * per;
    if (a >= n) break;
    const size_t len = std::min(per, n - a);
    th.emplace_back([=] { memcpy((uint8_t *)dst + a, (const uint8_t *)src + a, len); });
  }
  memcpy(dst, src, std::min(per, n));
  for (auto &x : th) x.join();
}
static bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  const bool ok = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
  (void)hipGetLastError(); // pageable memory reports an error: clear it
  return ok;
}
static bool stage_init(ymerge_ctx *c) {
  for (int k = 0; k < 2; k++) {
    if (!c->stage[k] && hipHostMalloc((void **)&c->stage[k], STAGE_CHUNK, hipHostMallocDefault) != hipSuccess)
      return false;
    if (!c->stage_ev[k] && hipEventCreateWithFlags(&c->stage_ev[k], hipEventDisableTiming) != hipSuccess)
      return false;
  }
  return true;
}
// host -> device on c->s; returns once the source may be reused
static bool copy_h2d(ymerge_ctx *c, void *dst, const void *src, size_t n) {
  if (!n) return true;
  if (n < STAGE_CHUNK / 4 || is_pinned(src) || !stage_init(c))
    return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->s) == hipSuccess &&
           hipStreamSynchronize(c->s) == hipSuccess;
  for (size_t off = 0, i = 0; off < n; off += STAGE_CHUNK, i++) {
    const int k = (int)(i & 1);
    const size_t len = std::min(STAGE_CHUNK, n - off);
    if (i >= 2 && hipEventSynchronize(c->stage_ev[k]) != hipSuccess) return false; // buffer k drained
    par_memcpy(c->stage[k], (const uint8_t *)src + off, len);
    if (hipMemcpyAsync((uint8_t *)dst + off, c->stage[k], len, hipMemcpyHostToDevice, c->s) != hipSuccess ||
        hipEventRecord(c->stage_ev[k], c->s) != hipSuccess)
      return false;
  }
  return hipStreamSynchronize(c->s) == hipSuccess;
}
// device -> host after the work queued on c->s; chunk k + 1's DMA overlaps chunk k's copy-out
static bool copy_d2h(ymerge_ctx *c, void *dst, const void *src, size_t n) {
  if (!n) return true;
  if (n < STAGE_CHUNK / 4 || is_pinned(dst) || !stage_init(c))
    return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->s) == hipSuccess;
  const size_t nch = (n + STAGE_CHUNK - 1) / STAGE_CHUNK;
  auto issue = [&](size_t i) {
    const size_t off = i * STAGE_CHUNK, len = std::min(STAGE_CHUNK, n - off);
    return hipMemcpyAsync(c->stage[i & 1], (const uint8_t *)src + off, len, hipMemcpyDeviceToHost, c->s) ==
               hipSuccess &&
           hipEventRecord(c->stage_ev[i & 1], c->s) == hipSuccess;
  };
  if (!issue(0)) return false;
  for (size_t i = 0; i < nch; i++) {
    if (i + 1 < nch && !issue(i + 1)) return false;
    if (hipEventSynchronize(c->stage_ev[i & 1]) != hipSuccess) return false;
    const size_t off = i * STAGE_CHUNK;
    par_memcpy((uint8_t *)dst + off, c->stage[i & 1], std::min(STAGE_CHUNK, n - off));
    // buffer (i & 1) is reused by chunk i + 2, issued after this copy-out
  }
  return true;
}

// grow `b` to `bytes` keeping its first `keep` bytes (device-to-device copy)
static bool ensure_keep(ymerge_ctx *c, DevBuf &b, size_t bytes, size_t keep) {
  if (bytes <= b.cap && b.p) return true;
  DevBuf nb;
  if (!nb.ensure(bytes)) return false;
  if (keep && b.p && hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, c->s) != hipSuccess) return false;
  if (hipStreamSynchronize(c->s) != hipSuccess) return false;
  b.release();
  b = nb;
  return true;
}

// fewest documents handed to k_fast_merge for its tiny-document hand-over to the exact engine
constexpr uint64_t TINY_MIN_DOCS = 262144;

// Documents per wavefront of the exact engine (ymerge_seq.hip): 64 (env YMERGE_SEQ_LPW sets it).
// One per wavefront was measured slower on the corpus (exact stage 2.35 vs 1.80 ms, r05t): the
// slowest document's serial walk sets the stage time either way, and 64 to a wave keeps the
// launch small.
static uint32_t seq_lpw(const ymerge_ctx *c, uint64_t n) {
  (void)n;
  return c->seq_lpw ? c->seq_lpw : 64;
}

// overflow words for the long updates k_decode_huge decodes (5 per block, 2 per DeleteSet entry,
// 3 per range: at most ~2.5 words per input byte, <= 2 on every realistic input; a batch that needs more leaves the rest on
// the merge kernels' walk)
static uint32_t huge_words(uint64_t n_bytes) { return (uint32_t)std::min<uint64_t>(2 * n_bytes + 65536, 1u << 26); }

// Scratch of the parallel long-update parse, sized from the batch's bytes (long updates total at
// most n_bytes; past LP_PMAX positions the rest take the exact walk).  Null when disabled or the
// allocation fails (then every long update takes the exact walk).
constexpr uint64_t LP_PMAX = 16u << 20;
static const ym::LpArgs *lp_args(ymerge_ctx *c, uint64_t n_bytes, uint32_t v1x) {
  static thread_local ym::LpArgs a;
  if (!c->long_parse) return nullptr;
  const uint64_t pcap = std::min<uint64_t>(n_bytes + 16, LP_PMAX);
  const uint64_t ccap = pcap / ym::LP_CH + ym::HUGE_LIST, scap = 4 * ccap + 65536, seccap = pcap / 3 + 16,
                 ocap = pcap / 2 + ym::HUGE_LIST, tcap = pcap / ym::LP_EXT_T + ym::HUGE_LIST;
  const uint64_t tmp = ym::scan_tmp_elems((uint32_t)ocap) + 2;
  const uint64_t bytes = 64ull * ym::HUGE_LIST + 64 + 4 * ccap + 4 * pcap + 8 * pcap + 4 * ym::LP_SEGW * scap +
                         16 * seccap + 8 * ocap + 8 * (ocap + 1) + 4 * ocap + 8ull * ym::HUGE_LIST + 8 * tmp + 8 * tcap + 512;
  if (!c->lp.ensure(bytes)) {
    (void)hipGetLastError();
    return nullptr;
  }
  uint8_t *q = c->lp.as<uint8_t>();
  auto take = [&](uint64_t n) {
    uint8_t *r = q;
    q += (n + 15) & ~15ull;
    return r;
  };
  a = ym::LpArgs{};
  a.meta = (uint32_t *)take(4ull * ym::LP_MW * ym::HUGE_LIST);
  a.g = (uint32_t *)take(4 * ym::LPG_WORDS);
  a.c2e = (uint32_t *)take(4 * ccap);
  a.ext = (uint32_t *)take(4 * pcap);
  a.jc = (uint64_t *)take(8 * pcap);
  a.seg = (uint32_t *)take(4 * ym::LP_SEGW * scap);
  a.sec = (uint32_t *)take(16 * seccap);
  a.blen = (uint64_t *)take(8 * ocap);
  a.sblen = (uint64_t *)take(8 * (ocap + 1));
  a.omap = (uint32_t *)take(4 * ocap);
  a.fb = (uint64_t *)take(8ull * ym::HUGE_LIST);
  a.scan_tmp = (uint64_t *)take(8 * tmp);
  a.tmap = (uint64_t *)take(8 * tcap);
  a.pcap = (uint32_t)pcap;
  a.ccap = (uint32_t)ccap;
  a.scap = (uint32_t)scap;
  a.seccap = (uint32_t)seccap;
  a.ocap = (uint32_t)ocap;
  a.tcap = (uint32_t)tcap;
  a.v1x = v1x;
  a.mid = c->lp_mid;
  return &a;
}

// Stage times of a merge whose documents were all written by k_lean: its one host round trip
// (hand-over count and output bytes) is taken right after k_lean, so the events recorded after
// it are read here -- by the stats getter, or before the next call records the events again --
// instead of in a second synchronisation per batch.
static void resolve_times(ymerge_ctx *c) {
  if (!c->times_pending) return;
  c->times_pending = false;
  if (hipEventSynchronize(c->ev[3]) != hipSuccess) return;
  float t70 = 0, t03 = 0;
  hipEventElapsedTime(&t70, c->ev[7], c->ev[0]);
  hipEventElapsedTime(&t03, c->ev[7], c->ev[3]);
  c->stats.ms_lean = t70;
  c->stats.ms_total = t03;
}

// One long single-client document over the whole GPU (ygiant.hip), queued without a host
// round trip: buffers are sized from host-known bounds (updates, bytes), the kernels read the
// counts they produce on the device, and k_gs_final leaves the document on path 2 (tiled kernel)
// when it is not that shape or outgrows a bound.  The deleted-clock bitmap holds one bit per input
// byte (at least 2^20: a clock unit of text is a byte of it), the squashed ranges one per 2 input
// bytes.
// run_giant's buffers (allocated before a graph capture: no allocation inside one)
static bool giant_ensure(ymerge_ctx *c, uint32_t U, uint64_t doc_bytes) {
  const size_t nu = (size_t)U + 1;
  const uint64_t nwc = std::min<uint64_t>(std::max<uint64_t>(doc_bytes / 32 + 2, 32768), 1ull << 26);
  const size_t nw = nwc, kc = (size_t)std::min<uint64_t>(nwc * 16, doc_bytes / 2 + 2) + 2;
  const size_t nparts = ((size_t)U + 255) / 256;
  return c->gs1.ensure((4 * nu + 8) * 8 + nparts * 28 + 64) &&
         c->scan_tmp.ensure(ym::scan_tmp_elems((uint32_t)std::max<size_t>(std::max<size_t>(nu, nw), kc)) * 8 + 64) &&
         c->gs2.ensure(nw * 4 + (2 * nw + 1) * 8 + 2 * kc * 4 + 2 * kc * 8 + 64);
}
static int run_giant(ymerge_ctx *c, const ym::BatchIn &b, const ym::FastOut &fo, uint32_t d, uint32_t U, uint64_t u0,
                     uint64_t doc_bytes) {
  ym::GsArgs a{};
  a.bytes = b.bytes;
  a.upd_off = b.upd_off;
  a.rec = b.rec;
  a.ovf = b.ovf;
  a.u0 = u0;
  a.U = U;
  a.d = d;
  a.out = fo.out;
  const size_t nu = (size_t)U + 1;
  const uint64_t nwc = std::min<uint64_t>(std::max<uint64_t>(doc_bytes / 32 + 2, 32768), 1ull << 26);
  a.nwords = (uint32_t)nwc;
  a.nbits = (uint32_t)((nwc - 2) * 32);
  a.kcap = (uint32_t)std::min<uint64_t>(nwc * 16, doc_bytes / 2 + 2);
  const size_t nw = a.nwords, kc = (size_t)a.kcap + 2;
  if (!giant_ensure(c, U, doc_bytes)) return DEV_FAIL();
  uint64_t *w = c->gs1.as<uint64_t>();
  a.cnt = w;
  a.bl = w + nu;
  a.s_cnt = w + 2 * nu;
  a.s_bl = w + 3 * nu;
  a.g = (uint32_t *)(w + 4 * nu);
  a.gp = a.g + 16; // (GS_WORDS)
  uint8_t *q = c->gs2.as<uint8_t>();
  a.w_cnt = (uint64_t *)q;
  a.w_scan = a.w_cnt + nw;
  a.k_size = a.w_scan + nw + 1;
  a.k_off = a.k_size + kc;
  a.bm = (uint32_t *)(a.k_off + kc);
  a.k_start = a.bm + nw;
  a.k_len = a.k_start + kc;
  // (no memsets: k_gs_pre zeroes the bitmap, k_gs_reduce / k_gs_write / k_gs_comp write g)
  ym::launch_gs_pre(a, c->s);
  ym::launch_scan_u64(a.cnt, a.s_cnt, U, c->scan_tmp.as<uint64_t>(), c->s);
  ym::launch_scan_u64(a.bl, a.s_bl, U, c->scan_tmp.as<uint64_t>(), c->s);
  ym::launch_gs_rest(a, fo, c->scan_tmp.as<uint64_t>(), c->s);
  return hipGetLastError() == hipSuccess ? 0 : DEV_FAIL();
}

// Single long update documents (ylong.hip): list entries read back from the device (LS_EW words:
// doc, update, L, NB, NE, NR, overflow word).  Scratch per document: 16 words, block sizes and
// offsets, range sizes and offsets, the scan's tiles; `scr_words` sums them for a list.
struct LsEntry {
  uint32_t d, L, NB, NE, NR, ovf;
  uint64_t u;
};
static uint64_t ls_scratch_words(const LsEntry &e) {
  return 16 + 2 * (2ull * e.NB + 2 + 4ull * e.NR + 4 + ym::scan_tmp_elems(std::max(e.NB, e.NR)) + 2 + e.NR + 1) + 16;
}
static std::vector<LsEntry> ls_entries(const uint32_t *w) {
  std::vector<LsEntry> v;
  const uint32_t n = std::min(w[0], ym::LS_LIST);
  for (uint32_t k = 0; k < n; k++) {
    const uint32_t *e = w + 4 + ym::LS_EW * k;
    v.push_back(LsEntry{e[0], e[3], e[4], e[5], e[6], e[7], e[1] | ((uint64_t)e[2] << 32)});
  }
  return v;
}
static void ls_bind(ym::LsArgs &a, const LsEntry &e, uint32_t *scr) {
  a.L = e.L;
  a.NB = e.NB;
  a.NE = e.NE;
  a.NR = e.NR;
  a.d = e.d;
  a.u = e.u;
  a.g = scr;
  uint64_t *q = (uint64_t *)(scr + 16);
  a.bsz = q;
  a.boff = q + e.NB;
  a.rsz = a.boff + e.NB + 2;
  a.roff = a.rsz + e.NR;
  a.rsz2 = a.roff + e.NR + 2;
  a.roff2 = a.rsz2 + e.NR;
  a.scan_tmp = a.roff2 + e.NR + 2;
  a.rstart = (uint32_t *)(a.scan_tmp + ym::scan_tmp_elems(std::max(e.NB, e.NR)) + 2);
  a.rend = a.rstart + e.NR;
}

// One batch: fast path for every document, exact engine for the documents it hands over.
// k_lean_fin's signal (lean_spin): host-mapped coherent words, allocated on first use
static bool ensure_sig(ymerge_ctx *c) {
  if (c->h_sig) return true;
  if (hipHostMalloc((void **)&c->h_sig, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    (void)hipGetLastError();
    c->h_sig = nullptr;
    return false;
  }
  memset(c->h_sig, 0, 4096);
  if (hipHostGetDevicePointer((void **)&c->d_sig, c->h_sig, 0) != hipSuccess) {
    (void)hipGetLastError();
    hipHostFree(c->h_sig);
    c->h_sig = nullptr;
    return false;
  }
  return true;
}
// poll for sequence number `seq` (written last by k_lean_fin); the stream is queried now and
// then so that a failed kernel ends the wait
static bool wait_sig(ymerge_ctx *c, uint32_t seq) {
  const volatile uint32_t *f = c->h_sig;
  for (uint64_t it = 1;; it++) {
    if (*f == seq) break;
    if ((it & 4095) == 0) {
      const hipError_t e = hipStreamQuery(c->s);
      if (e == hipSuccess) {
        if (*f == seq) break;
        return false; // the stream drained without the signal
      }
      if (e != hipErrorNotReady) return false;
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return true;
}

static int merge_device(ymerge_ctx *c, const uint8_t *d_bytes, uint64_t n_bytes, const uint64_t *d_upd_off,
                        uint64_t n_updates, const uint64_t *d_doc_upd, uint64_t n_docs, ymerge_device_result *res) {
  resolve_times(c);
  if (hipSetDevice(c->device) != hipSuccess) return DEV_FAIL();
  if (n_docs > 0xFFFFFFFFull) return YMERGE_ERR_OTHER;
  const uint32_t n = (uint32_t)n_docs;
  ym::BatchIn b{d_bytes, d_upd_off, d_doc_upd, n, nullptr, nullptr};
  b.v1x = d_bytes == c->v2x.as<uint8_t>(); // the lib0 v2 path's transcoded arena
  const size_t nn = (size_t)n + 1;
  const uint64_t slots = 2 * n_bytes + 64 * (uint64_t)n_docs;
  if (!c->status.ensure(nn) || !c->path.ensure(nn) || !c->out_start.ensure(nn * 8) || !c->out_len.ensure(nn * 8) ||
      !c->pack_off.ensure(nn * 8) || !c->counts.ensure(4 * nn * 4) || !c->need.ensure(nn * 8) ||
      !c->scr_off.ensure(nn * 8) || !c->sizes.ensure(nn * 8) || !c->spill_off.ensure(nn * 8) ||
      !c->scan_tmp.ensure(ym::scan_tmp_elems(n) * 8 + 64) || !c->counter.ensure(128 + 64 * 64) ||
      !ensure_keep(c, c->arena, slots + slots / 8 + 4096, 0) ||
      (c->fast_threads && (!c->rec.ensure((n_updates + 1) * ym::REC_WORDS * 4) ||
                           !c->ovf.ensure(((n_updates + ym::DEC_NT - 1) / ym::DEC_NT + 1) * ym::DEC_OVF * 4 +
                                          (uint64_t)huge_words(n_bytes) * 4) ||
                           !c->huge.ensure(ym::huge_bytes(n_updates)))))
    return DEV_FAIL();
  b.rec = c->rec.as<uint32_t>();
  b.ovf = c->ovf.as<uint32_t>();
  uint8_t *arena = c->arena.as<uint8_t>();
  uint64_t *ostart = c->out_start.as<uint64_t>(), *olen = c->out_len.as<uint64_t>();
  uint8_t *status = c->status.as<uint8_t>(), *path = c->path.as<uint8_t>();
  // counters [128 B] then k_lean's 64 output-byte partial sums [4 KB]: one memset, one copy back
  // (none when the last merge ended in k_lean_fin, which zeroes them after reading)
  if (c->counters_clean != c->counter.p) hipMemsetAsync(c->counter.p, 0, 128 + 64 * 64, c->s);
  c->counters_clean = nullptr;
  uint64_t *stamps = nullptr;
  if (c->want_stamps) {
    if (!c->stamps.ensure(nn * 16 * 8)) return DEV_FAIL();
    hipMemsetAsync(c->stamps.p, 0, nn * 16 * 8, c->s);
    stamps = c->stamps.as<uint64_t>();
    c->stamps_docs = n_docs;
  }
  if (!c->big_list.ensure(nn * 4)) return DEV_FAIL();
  ym::FastOut fo{arena, ostart, olen, status, path, stamps, nullptr, c->counter.as<uint32_t>() + 4};
  fo.big_list = c->big_list.as<uint32_t>();
  if (getenv("YMERGE_LEAN_DEBUG") && c->lean_dbg.ensure(nn * 32)) {
    hipMemsetAsync(c->lean_dbg.p, 0xFF, nn * 32, c->s);
    fo.dbg = c->lean_dbg.as<uint32_t>();
  }
  (void)hipGetLastError(); // a failed optional allocation must not fail the launches below
  // k_lean: one wavefront per document for the common shape; the rest (path 3) goes on to
  // k_decode + k_fast_merge, which are skipped when k_lean wrote every document
  const bool lean = c->lean && c->fast_threads;
  uint32_t n_rej = n;
  // One long document alone in the batch (C1: an editing trace as per-op updates): k_decode,
  // then the grid-wide kernels, with one host round trip at the end instead of the hand-over
  // reads of k_lean, k_fast_merge and the listing.  Not that shape: the batch takes the
  // general route below, which keeps the records and does not list the document for the grid
  // path again (that second attempt failed the same way).
  bool decoded = false, giant_rejected = false;
  // grid-path threshold of this batch: lower for a batch of few documents (ykernels.h)
  const uint32_t gmin = c->giant_min && n <= ym::GS_SMALL_DOCS ? std::min(c->giant_min, ym::GS_MIN_SMALL) : c->giant_min;
  if (n == 1 && gmin && n_updates >= gmin && n_updates < (1ull << 31) && c->fast_threads &&
      !c->want_stamps && c->giant_lane) {
    hipEventRecord(c->ev[7], c->s);
    const ym::LpArgs *la = lp_args(c, n_bytes, b.v1x);
    if (!giant_ensure(c, (uint32_t)n_updates, n_bytes)) return DEV_FAIL();
    // the launch sequence's key: inputs, buffer addresses, grammar, parse settings
    uint64_t key = 0xcbf29ce484222325ull;
    auto mix = [&](uint64_t v) { key = (key ^ v) * 0x100000001b3ull; };
    for (uint64_t v : {(uint64_t)d_bytes, n_bytes, (uint64_t)d_upd_off, n_updates, (uint64_t)d_doc_upd,
                       (uint64_t)b.v1x, (uint64_t)c->rec.p, (uint64_t)c->ovf.p, (uint64_t)c->huge.p,
                       (uint64_t)c->lp.p, (uint64_t)c->gs1.p, (uint64_t)c->gs2.p, (uint64_t)c->scan_tmp.p,
                       (uint64_t)arena, (uint64_t)ostart, (uint64_t)olen, (uint64_t)status, (uint64_t)path,
                       (uint64_t)c->counter.p, (uint64_t)(la != nullptr), (uint64_t)c->lp_mid})
      mix(v);
    bool graphed = false;
    if (c->giant_graph && c->giant_exec && c->graph_key == key) {
      graphed = hipGraphLaunch(c->giant_exec, c->s) == hipSuccess;
    } else if (c->giant_graph && c->giant_key == key &&
               hipStreamBeginCapture(c->s, hipStreamCaptureModeThreadLocal) == hipSuccess) {
      ym::launch_decode(d_bytes, d_upd_off, n_updates, c->rec.as<uint32_t>(), c->ovf.as<uint32_t>(),
                        c->huge.as<uint32_t>(), huge_words(n_bytes), c->s, la, b.v1x);
      const int rc0 = run_giant(c, b, fo, 0, (uint32_t)n_updates, 0, n_bytes);
      hipGraph_t g = nullptr;
      const hipError_t ec = hipStreamEndCapture(c->s, &g);
      if (ec == hipSuccess && rc0 == 0 && g) {
        if (c->giant_exec) hipGraphExecDestroy(c->giant_exec);
        c->giant_exec = nullptr;
        if (hipGraphInstantiate(&c->giant_exec, g, nullptr, nullptr, 0) == hipSuccess) {
          c->graph_key = key;
          graphed = hipGraphLaunch(c->giant_exec, c->s) == hipSuccess;
        } else {
          c->giant_exec = nullptr;
        }
      }
      if (g) hipGraphDestroy(g);
      (void)hipGetLastError();
      if (!graphed) c->giant_graph = false; // capture not usable here: eager from now on
    }
    if (!graphed) { // eager launches (the first run of a key, or graphs off)
      hipEventRecord(c->ev[0], c->s);
      ym::launch_decode(d_bytes, d_upd_off, n_updates, c->rec.as<uint32_t>(), c->ovf.as<uint32_t>(),
                        c->huge.as<uint32_t>(), huge_words(n_bytes), c->s, la, b.v1x); // (no probe: one sync less)
      hipEventRecord(c->ev[5], c->s);
      const int rc = run_giant(c, b, fo, 0, (uint32_t)n_updates, 0, n_bytes);
      if (rc) return rc;
      c->giant_key = key;
    }
    decoded = true;
    hipEventRecord(c->ev[1], c->s);
    hipMemcpyAsync(c->h_pinned + 20, path, 1, hipMemcpyDeviceToHost, c->s);
    hipMemcpyAsync(c->h_pinned + 21, olen, 8, hipMemcpyDeviceToHost, c->s);
    if (hipStreamSynchronize(c->s) != hipSuccess) return DEV_FAIL();
    if ((c->h_pinned[20] & 0xFF) == 0) {
      float t05 = 0, t51 = 0, t71 = 0;
      hipEventElapsedTime(&t71, c->ev[7], c->ev[1]);
      if (graphed) { // (one graph: no split between decode and the grid kernels)
        t51 = t71;
      } else {
        hipEventElapsedTime(&t05, c->ev[0], c->ev[5]);
        hipEventElapsedTime(&t51, c->ev[5], c->ev[1]);
      }
      c->stats = ymerge_stats{};
      c->stats.n_docs = n_docs;
      c->stats.bytes_in = n_bytes;
      c->stats.bytes_out = c->h_pinned[21];
      c->stats.docs_big = 1;
      c->stats.docs_giant = 1;
      c->stats.ms_decode = t05;
      c->stats.ms_big = t51;
      c->stats.ms_total = t71;
      c->pack_stale = true; // pack_off is the one document's length: computed when a host copy asks
      res->d_out = arena;
      res->d_out_start = ostart;
      res->d_out_len = olen;
      res->d_status = status;
      res->arena_bytes = c->arena.cap;
      res->out_bytes = c->h_pinned[21];
      return 0;
    }
    giant_rejected = true; // k_gs_final left it on path 2: the general route takes it
  }
  const bool no_ev = !c->timing; // (ymerge_ctx_set_stage_timing)
  if (!no_ev) hipEventRecord(c->ev[7], c->s);
  if (lean) {
    // BIG k_lean documents keep their size-proportional tables in HBM (untouched otherwise)
    const uint64_t lw = ym::lean_scratch_words(n_updates, n_docs, n_bytes);
    // without it k_lean hands its BIG documents over (path 3) instead of failing the batch;
    // the failed hipMalloc's sticky error is cleared so the launch check below stays meaningful
    uint32_t *lscr = nullptr;
    if (lw * 4 + 64 <= c->lean_scr_max && c->lean_scr.ensure(lw * 4 + 64)) lscr = c->lean_scr.as<uint32_t>();
    (void)hipGetLastError();
    fo.lean_total = (unsigned long long *)(c->counter.as<uint8_t>() + 128);
    // large batches: long documents dispatched first (a skewed batch otherwise ends on the
    // last long document to start)
    ym::BatchIn bl = b;
    if (gmin && n <= ym::GS_SMALL_DOCS) bl.lean_umax = gmin - 1; // (documents of >= gmin updates: grid path or tiled)
    // (batches of many small documents: Zipf-like tenants, where one long document would
    // otherwise end the kernel; also the ~48 MB groups of the pipelined host entry)
    if (c->lean_order == 1 || (c->lean_order < 0 && n >= 8192 && n_updates < 256ull * n)) {
      if (!c->lean_ord.ensure((size_t)n * 4 + 64)) return DEV_FAIL();
      hipMemsetAsync(c->lean_ord.p, 0, 64, c->s); // class counts and cursors (<= 16 words)
      ym::launch_lean_order(d_doc_upd, n, c->lean_ord.as<uint32_t>(), c->lean_ord.as<uint32_t>() + 16, c->s);
      bl.order = c->lean_ord.as<uint32_t>() + 16;
    }
    ym::launch_lean(bl, fo, lscr, c->s);
    if (hipGetLastError() != hipSuccess) return DEV_FAIL();
    // k_lean's end (ms_lean = ev7 -> ev0: the kernel, not the host's turnaround after it; the
    // general route records ev0 again below)
    if (!no_ev) hipEventRecord(c->ev[0], c->s);
    if (c->lean_spin && ensure_sig(c)) {
      // hand-over count and output bytes summed by k_lean_fin into the host-mapped words
      const uint32_t seq = ++c->sig_seq ? c->sig_seq : ++c->sig_seq;
      ym::launch_lean_fin(c->counter.as<uint32_t>(), c->d_sig, seq, c->s);
      if (!no_ev) hipEventRecord(c->ev[3], c->s); // (the end of a merge that k_lean writes whole)
      if (hipGetLastError() != hipSuccess || !wait_sig(c, seq)) return DEV_FAIL();
      c->h_pinned[501] = c->h_sig[1];
      for (int q = 0; q < 64; q++) c->h_pinned[512 + 8 * q] = 0;
      c->h_pinned[512] = (uint64_t)c->h_sig[2] | ((uint64_t)c->h_sig[3] << 32);
      if (c->h_pinned[501] == 0) c->counters_clean = c->counter.p; // (the other paths update them next)
    } else {
      // hand-over count and k_lean's output bytes (npath[6] at counter byte 40, the 64 partial
      // sums from byte 128) in one copy and one sync: byte 128 lands on h_pinned[512]
      hipMemcpyAsync((uint8_t *)(c->h_pinned + 512) - 88, c->counter.as<uint8_t>() + 40, 88 + 64 * 64,
                     hipMemcpyDeviceToHost, c->s);
      if (hipStreamSynchronize(c->s) != hipSuccess) return DEV_FAIL();
      uint32_t sh = 0; // the hand-over shards: word 2 of each 64-byte partial
      for (int q = 0; q < 64; q++) sh += (uint32_t)c->h_pinned[512 + 8 * q + 1];
      c->h_pinned[501] = (uint32_t)c->h_pinned[501] + sh;
    }
    n_rej = (uint32_t)(c->h_pinned[501] & 0xFFFFFFFFu);
    b.only_path3 = 1;
    if (n_rej && getenv("YMERGE_LEAN_DEBUG")) {
      uint32_t why[7];
      hipMemcpy(why, c->counter.as<uint32_t>() + 11, sizeof why, hipMemcpyDeviceToHost);
      fprintf(stderr, "k_lean handed over %u/%u docs: size %u stage %u walk %u clients %u arena %u contiguity %u window %u\n",
              n_rej, n, why[0], why[1], why[2], why[3], why[4], why[5], why[6]);
      std::vector<uint32_t> g(8 * (size_t)n);
      hipMemcpy(g.data(), fo.dbg, g.size() * 4, hipMemcpyDeviceToHost);
      for (uint32_t q = 0, shown = 0; q < n && shown < 4; q++)
        if (g[8 * q] != 0xFFFFFFFFu) {
          fprintf(stderr, "  doc %u: lane %u clock %u prevl %d exp0 %u pend %u bk %u end0 %u ub %u\n", q, g[8 * q],
                  g[8 * q + 1], (int)g[8 * q + 2], g[8 * q + 3], g[8 * q + 4], g[8 * q + 5], g[8 * q + 6], g[8 * q + 7]);
          shown++;
        }
    }
  }
  if (!lean || n_rej) hipEventRecord(c->ev[0], c->s);
  const bool fast = c->fast_threads && n_rej > 0;
  if (fast) {
    // diagnostic (env YMERGE_DECODE_DBG): k_decode_exact's slowest workgroups to stderr
    static const bool ddbg = getenv("YMERGE_DECODE_DBG") != nullptr;
    const uint64_t nwg = (n_updates + ym::DEC_NT - 1) / ym::DEC_NT;
    uint64_t *dbg = nullptr;
    if (ddbg && c->stamps.ensure(nwg * 64 + 64)) {
      hipMemsetAsync(c->stamps.p, 0, nwg * 64, c->s);
      dbg = c->stamps.as<uint64_t>();
    }
    if (!decoded) // (the grid lane's records are still valid)
      ym::launch_decode(d_bytes, d_upd_off, n_updates, c->rec.as<uint32_t>(), c->ovf.as<uint32_t>(),
                        c->huge.as<uint32_t>(), huge_words(n_bytes), c->s, lp_args(c, n_bytes, b.v1x), b.v1x, dbg,
                        (uint32_t *)(c->h_pinned + 24));
    if (dbg) {
      std::vector<uint64_t> h(nwg * 8);
      hipStreamSynchronize(c->s);
      hipMemcpy(h.data(), dbg, nwg * 64, hipMemcpyDeviceToHost);
      std::vector<size_t> idx(nwg);
      for (size_t q = 0; q < nwg; q++) idx[q] = q;
      std::sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return h[8 * x + 3] > h[8 * y + 3]; });
      for (size_t q = 0; q < std::min<size_t>(8, nwg); q++) {
        const uint64_t *o = h.data() + 8 * idx[q];
        fprintf(stderr, "k_decode_exact tile %lu: pending %lu rounds %lu cycles %lu slowest walk %lu (update %lu) bytes %lu\n",
                (unsigned long)o[0], (unsigned long)o[1], (unsigned long)o[2], (unsigned long)o[3], (unsigned long)(o[7] >> 24),
                (unsigned long)(o[7] & 0xFFFFFF), (unsigned long)o[6]);
      }
    }
    hipEventRecord(c->ev[5], c->s);
    // the tiny-document hand-over pays off only for many of them (C3: 645k documents of <= 4
    // updates, 13.5 -> 4.5 ms): the exact engine's lane walks chase HBM scratch (~1 ms a
    // wavefront of 64 tiny documents), a fast-path workgroup takes one in ~40 us
    ym::FastCaps caps = c->caps;
    if (n_rej < TINY_MIN_DOCS && !c->tiny_forced) caps.in_cap = 0;
    ym::launch_fast_merge(b, caps, fo, c->fast_threads, c->s);
    if (hipGetLastError() != hipSuccess) return DEV_FAIL();
    hipEventRecord(c->ev[6], c->s);
  }
  else {
    hipEventRecord(c->ev[5], c->s);
    hipEventRecord(c->ev[6], c->s);
    if (!c->fast_threads) hipMemsetAsync(path, 1, n, c->s);
  }
  // hand-over counts of the fast path (npath[1] exact engine, npath[2] tiled kernel): the
  // later stages are skipped when no document needs them
  uint32_t n_p1 = c->fast_threads ? 0 : n, n_p2 = 0;
  if (fast) {
    hipMemcpyAsync(c->h_pinned + 12, c->counter.as<uint32_t>() + 4, 16, hipMemcpyDeviceToHost, c->s);
    if (hipStreamSynchronize(c->s) != hipSuccess) return DEV_FAIL();
    const uint32_t *np = (const uint32_t *)(c->h_pinned + 12);
    n_p1 = np[1];
    n_p2 = np[2];
  }
  // documents over the LDS capacities (path == 2): count, scratch offsets, tiled kernel
  uint32_t n_big = 0;
  if (fast && n_p2) {
    // long single-client documents first (ygiant.hip): listed and marked GS_PATH, merged by the
    // grid-wide kernels; the ones that are not that shape return to path 2 before k_big_count
    const bool giant = gmin && n_updates >= gmin && !c->want_stamps && !giant_rejected;
    // single long update documents (one REC_LONG record, ylong.hip): listed in the same round trip
    const bool lsg = c->long_parse && c->long_grid && !c->want_stamps;
    constexpr size_t GSL = 1 + 6 * ym::GS_LIST, LSL = 4 + ym::LS_EW * ym::LS_LIST;
    if (giant || lsg) {
      if (!c->gs_list.ensure(GSL * 8) || !c->ls_list.ensure(LSL * 4)) return DEV_FAIL();
      if (giant) {
        hipMemsetAsync(c->gs_list.p, 0, 8, c->s);
        ym::launch_gs_find(b, path, gmin, c->gs_list.as<uint64_t>(), c->s);
        hipMemcpyAsync(c->h_pinned + 128, c->gs_list.p, GSL * 8, hipMemcpyDeviceToHost, c->s);
      }
      if (lsg) {
        hipMemsetAsync(c->ls_list.p, 0, 16, c->s);
        ym::launch_ls_find(b, path, c->ls_list.as<uint32_t>(), c->s);
        hipMemcpyAsync(c->h_pinned + 256, c->ls_list.p, LSL * 4, hipMemcpyDeviceToHost, c->s);
      }
      if (hipStreamSynchronize(c->s) != hipSuccess) return dev_err("long-document listing");
    }
    if (giant) {
      uint64_t ent[GSL];
      memcpy(ent, c->h_pinned + 128, sizeof ent);
      const uint64_t ng = std::min<uint64_t>(ent[0], ym::GS_LIST);
      for (uint64_t k = 0; k < ng; k++) { // e = (document, updates, ranges, first update, first byte, bytes)
        const uint64_t *e = ent + 1 + 6 * k;
        const int rc = run_giant(c, b, fo, (uint32_t)e[0], (uint32_t)e[1], e[3], e[5]);
        if (rc) return rc;
      }
    }
    if (lsg) {
      const std::vector<LsEntry> ls = ls_entries((const uint32_t *)(c->h_pinned + 256));
      uint64_t words = 0;
      for (const LsEntry &e : ls) words = std::max(words, ls_scratch_words(e));
      if (!ls.empty() && !c->ls_scr.ensure(words * 4 + 64)) return DEV_FAIL();
      for (const LsEntry &e : ls) { // one after the other on the stream: the scratch is reused
        ym::LsArgs a{};
        a.bytes = b.bytes;
        a.upd_off = b.upd_off;
        a.ov = b.ovf + e.ovf;
        a.mode = 0;
        a.v1x = b.v1x;
        a.out = fo.out;
        a.out_start = fo.out_start;
        a.out_len = fo.out_len;
        a.status = fo.status;
        a.path = fo.path;
        a.npath = fo.npath;
        ls_bind(a, e, c->ls_scr.as<uint32_t>());
        ym::launch_ls_doc(a, 0, c->s);
      }
      if (hipGetLastError() != hipSuccess) return dev_err("long-document merge launch");
    }
    hipMemsetAsync(c->need.p, 0, (size_t)n * 8, c->s); // (k_big_count writes the listed documents' words)
    ym::launch_big_count(b, fo, c->counts.as<uint32_t>(), c->need.as<uint64_t>(), c->counter.as<uint32_t>() + 2, n_p2,
                         c->s);
    ym::launch_scan_u64(c->need.as<uint64_t>(), c->scr_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
    hipMemcpyAsync(c->h_pinned + 10, c->scr_off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, c->s);
    hipMemcpyAsync(c->h_pinned + 11, c->counter.as<uint32_t>() + 2, 4, hipMemcpyDeviceToHost, c->s);
    if (hipStreamSynchronize(c->s) != hipSuccess) return DEV_FAIL();
    n_big = (uint32_t)(c->h_pinned[11] & 0xFFFFFFFFu);
    if (n_big) {
      if (!c->big_scratch.ensure((size_t)c->h_pinned[10] * 4 + 64)) return DEV_FAIL();
      ym::launch_big_merge(b, c->counts.as<uint32_t>(), c->scr_off.as<uint64_t>(), c->big_scratch.as<uint32_t>(), fo,
                           n_p2, c->s);
      if (hipGetLastError() != hipSuccess) return DEV_FAIL();
    }
  }
  hipEventRecord(c->ev[1], c->s);
  // exact engine for documents the fast or tiled path handed over (path == 1)
  uint64_t words = 0;
  uint32_t n_exact = 0, n_overlap = 0, n_tiny = 0, n_giant = 0;
  if (n_p1 || n_p2) {
    ym::launch_seq_count(b, path, status, c->counts.as<uint32_t>(), c->need.as<uint64_t>(), c->counter.as<uint32_t>(),
                         c->s, seq_lpw(c, fast ? (uint64_t)n_p1 + n_p2 : n));
    ym::launch_scan_u64(c->need.as<uint64_t>(), c->scr_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
    hipMemcpyAsync(c->h_pinned + 8, c->scr_off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, c->s);
    hipMemcpyAsync(c->h_pinned + 9, c->counter.p, 4, hipMemcpyDeviceToHost, c->s);
    hipMemcpyAsync(c->h_pinned + 14, c->counter.as<uint32_t>() + 7, 12, hipMemcpyDeviceToHost, c->s);
    hipMemcpyAsync(c->h_pinned + 17, c->counter.as<uint32_t>() + 18, 8, hipMemcpyDeviceToHost, c->s); // npath[14..15]
    if (hipStreamSynchronize(c->s) != hipSuccess) return DEV_FAIL();
    words = c->h_pinned[8];
    n_exact = (uint32_t)(c->h_pinned[9] & 0xFFFFFFFFu);
    n_overlap = (uint32_t)(c->h_pinned[14] & 0xFFFFFFFFu);
    n_big -= (uint32_t)(c->h_pinned[14] >> 32); // tiled-kernel documents handed to the exact engine
    n_tiny = (uint32_t)(c->h_pinned[15] & 0xFFFFFFFFu);
    n_giant = (uint32_t)(c->h_pinned[17] & 0xFFFFFFFFu) + (uint32_t)(c->h_pinned[17] >> 32); // + long-update grid path
  }
  if (n_exact) {
    if (!c->scratch.ensure((size_t)words * 4 + 64)) return DEV_FAIL();
    const uint32_t lpw = seq_lpw(c, n_exact);
    static const bool seq_dbg = getenv("YMERGE_SEQ_DBG") != nullptr;
    uint64_t *sdbg = nullptr;
    if (seq_dbg && c->stamps.ensure((size_t)n * 8 + 64)) {
      sdbg = c->stamps.as<uint64_t>();
      hipMemsetAsync(sdbg, 0, (size_t)n * 8, c->s);
    }
    ym::launch_seq_merge(false, b, path, status, c->counts.as<uint32_t>(), c->scr_off.as<uint64_t>(),
                         c->scratch.as<uint32_t>(), c->sizes.as<uint64_t>(), nullptr, nullptr, 0, nullptr, nullptr,
                         status, c->s, lpw);
    ym::launch_scan_u64(c->sizes.as<uint64_t>(), c->spill_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
    uint64_t spill = 0;
    if (!read_words(c, c->spill_off.as<uint64_t>() + n, 8, &spill)) return DEV_FAIL();
    if (!ensure_keep(c, c->arena, slots + spill + 4096, slots)) return DEV_FAIL();
    arena = c->arena.as<uint8_t>();
    ym::launch_seq_merge(true, b, path, status, c->counts.as<uint32_t>(), c->scr_off.as<uint64_t>(),
                         c->scratch.as<uint32_t>(), nullptr, c->spill_off.as<uint64_t>(), arena, slots, ostart, olen,
                         nullptr, c->s, lpw, sdbg);
    if (hipGetLastError() != hipSuccess) return DEV_FAIL();
    if (sdbg) { // diagnostic (env YMERGE_SEQ_DBG): the exact engine's slowest documents to stderr
      std::vector<uint64_t> h(n), du(n + 1);
      hipStreamSynchronize(c->s);
      hipMemcpy(h.data(), sdbg, n * 8, hipMemcpyDeviceToHost);
      hipMemcpy(du.data(), b.doc_upd, (n + 1) * 8, hipMemcpyDeviceToHost);
      std::vector<uint32_t> idx(n);
      for (uint32_t q = 0; q < n; q++) idx[q] = q;
      std::sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return h[x] > h[y]; });
      for (uint32_t q = 0; q < std::min<uint32_t>(8, n) && h[idx[q]]; q++) {
        uint64_t o0 = 0, o1 = 0;
        hipMemcpy(&o0, b.upd_off + du[idx[q]], 8, hipMemcpyDeviceToHost);
        hipMemcpy(&o1, b.upd_off + du[idx[q] + 1], 8, hipMemcpyDeviceToHost);
        fprintf(stderr, "k_seq_merge doc %u: updates %lu bytes %lu cycles %lu\n", idx[q],
                (unsigned long)(du[idx[q] + 1] - du[idx[q]]), (unsigned long)(o1 - o0), (unsigned long)h[idx[q]]);
      }
    }
  }
  // total output bytes (and packed offsets for host copies); when k_lean wrote every
  // document its byte counter is the total and the scan waits for a host copy (pack_to_host)
  uint64_t total = 0;
  c->pack_stale = lean && n_rej == 0;
  if (!c->pack_stale || !c->lean_spin || !c->h_sig) hipEventRecord(c->ev[2], c->s);
  if (c->pack_stale) {
    for (int q = 0; q < 64; q++) total += c->h_pinned[512 + 8 * q];
    if (!c->lean_spin || !c->h_sig) hipEventRecord(c->ev[3], c->s); // (else recorded after k_lean_fin)
    if (hipGetLastError() != hipSuccess) return DEV_FAIL();
    c->stats = ymerge_stats{};
    c->stats.n_docs = n_docs;
    c->stats.bytes_in = n_bytes;
    c->stats.docs_lean = n_docs;
    c->stats.bytes_out = total;
    c->times_pending = !no_ev; // ms_lean / ms_total: resolve_times
    res->d_out = arena;
    res->d_out_start = ostart;
    res->d_out_len = olen;
    res->d_status = status;
    res->arena_bytes = c->arena.cap;
    res->out_bytes = total;
    return 0;
  } else {
    ym::launch_scan_u64(olen, c->pack_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
    hipEventRecord(c->ev[3], c->s);
    if (!read_words(c, c->pack_off.as<uint64_t>() + n, 8, &total)) return DEV_FAIL();
  }
  if (hipGetLastError() != hipSuccess) return DEV_FAIL();
  float t01 = 0, t12 = 0, t23 = 0, t03 = 0, t05 = 0, t61 = 0, t70 = 0;
  hipEventElapsedTime(&t70, c->ev[7], c->ev[0]);
  hipEventElapsedTime(&t05, c->ev[0], c->ev[5]);
  hipEventElapsedTime(&t01, c->ev[5], c->ev[6]);
  hipEventElapsedTime(&t61, c->ev[6], c->ev[1]);
  hipEventElapsedTime(&t12, c->ev[1], c->ev[2]);
  hipEventElapsedTime(&t23, c->ev[2], c->ev[3]);
  hipEventElapsedTime(&t03, c->ev[7], c->ev[3]);
  c->stats = ymerge_stats{};
  c->stats.n_docs = n_docs;
  c->stats.bytes_in = n_bytes;
  c->stats.docs_lean = lean ? n_docs - n_rej : 0;
  c->stats.ms_lean = lean ? t70 : 0.0f;
  c->stats.bytes_out = total;
  c->stats.docs_exact = n_exact - n_tiny;
  c->stats.docs_tiny = n_tiny;
  c->stats.ms_tiny = n_exact == n_tiny ? t12 : 0.0f;
  c->stats.docs_big = n_big + n_giant; // grid-path documents leave path 2 before k_big_count
  c->stats.docs_overlap = n_overlap;
  c->stats.docs_giant = n_giant;
  c->stats.docs_fast = n_docs - n_exact - c->stats.docs_big - c->stats.docs_lean;
  c->stats.ms_big = t61;
  c->stats.ms_fast = t01;
  c->stats.ms_exact = t12;
  c->stats.ms_tail = t23;
  c->stats.ms_decode = t05;
  c->stats.ms_total = t03;
  res->d_out = arena;
  res->d_out_start = ostart;
  res->d_out_len = olen;
  res->d_status = status;
  res->arena_bytes = c->arena.cap;
  res->out_bytes = total;
  return 0;
}

extern "C" int ymerge_updates_v1_batch_device(ymerge_ctx *c, const uint8_t *d_bytes, uint64_t n_bytes,
                                              const uint64_t *d_upd_off, uint64_t n_updates, const uint64_t *d_doc_upd,
                                              uint64_t n_docs, ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return merge_device(c, d_bytes, n_bytes, d_upd_off, n_updates, d_doc_upd, n_docs, res);
}

// diff_updates_v1 / encode_state_vector_from_update_v1 over a batch (one update per document):
// plan (small scratch) -> re-plan the overflowing documents with length-sized scratch ->
// output offsets (scan) -> execute.
// frame: 0 plain, 1 y-sync SyncStep2 reply (diff; d_sv = client messages, parsed here),
// 2 y-sync SyncStep1 message (state vector)
static int plan_exec(ymerge_ctx *c, bool diff, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                     const uint8_t *d_sv, const uint64_t *d_sv_off, uint64_t n_docs, ymerge_device_result *res,
                     uint32_t frame = 0, const uint64_t *sv_end = nullptr, const uint8_t *pre_status = nullptr) {
  resolve_times(c);
  if (hipSetDevice(c->device) != hipSuccess) return DEV_FAIL();
  if (n_docs > 0xFFFFFFFFull) return YMERGE_ERR_OTHER;
  const uint32_t n = (uint32_t)n_docs;
  ym::DiffBatch b{d_bytes, d_upd_off, d_sv, d_sv_off, n};
  c->pack_stale = false; // pack_off = this batch's output offsets (set below)
  b.v1x = d_bytes == c->v2x.as<uint8_t>(); // the lib0 v2 path's transcoded arena
  b.frame = frame;
  if (frame == 1) {
    if (!c->sync_off.ensure((n + 1) * 8) || !c->sync_end.ensure((n + 1) * 8) || !c->sync_st.ensure(n + 1))
      return DEV_FAIL();
    ym::launch_sync_parse(d_sv, d_sv_off, n, c->sync_off.as<uint64_t>(), c->sync_end.as<uint64_t>(),
                          c->sync_st.as<uint8_t>(), c->s);
    b.sv_off = c->sync_off.as<uint64_t>();
    b.sv_end = c->sync_end.as<uint64_t>();
    b.pre_status = c->sync_st.as<uint8_t>();
  }
  if (pre_status) { // lib0 v2 front end: state-vector slices and decode statuses
    b.sv_end = sv_end;
    b.pre_status = pre_status;
  }
  const size_t nn = (size_t)n + 1;
  const uint64_t sw = ym::plan_small_words();
  if (!c->status.ensure(nn) || !c->path.ensure(nn) || !c->out_len.ensure(nn * 8) || !c->pack_off.ensure(nn * 8) ||
      !c->need.ensure(nn * 8) || !c->spill_off.ensure(nn * 8) || !c->scan_tmp.ensure(ym::scan_tmp_elems(n) * 8 + 64) ||
      !c->counter.ensure(64) || !c->plan_small.ensure(nn * sw * 4) || !c->plan_wlist.ensure(nn * 4))
    return DEV_FAIL();
  ym::PlanScratch ps{c->plan_small.as<uint32_t>(), sw,       nullptr,
                     c->spill_off.as<uint64_t>(), c->path.as<uint8_t>(), c->status.as<uint8_t>(),
                     c->out_len.as<uint64_t>(),    c->counter.as<uint32_t>()};
  ps.planner = c->planner;
  if (const char *v = getenv("YMERGE_LANE_DBG")) ps.lane_dbg = (uint32_t)atoi(v);
  ps.wave_list = c->plan_wlist.as<uint32_t>();
  ps.wave_n = c->counter.as<uint32_t>() + 8; // zeroed with the counters below
  if (c->want_stamps) { // diagnostic: k_plan_ring phase cycles
    if (!c->stamps.ensure(nn * 16 * 8)) return DEV_FAIL();
    hipMemsetAsync(c->stamps.p, 0, nn * 16 * 8, c->s);
    ps.stamps = c->stamps.as<uint64_t>();
    c->stamps_docs = n_docs;
  }
  hipMemsetAsync(c->counter.p, 0, 64, c->s);
  c->counters_clean = nullptr;
  hipEventRecord(c->ev[0], c->s);
  // documents of >= ls_min_diff bytes: the parallel long-update parse, then the grid path for the
  // single-section ones (ylong.hip); the planners skip what it takes (b.ls_done)
  std::vector<LsEntry> ls;
  std::vector<uint64_t> ls_off;
  if (c->long_parse && c->long_grid && c->ls_min_diff && !c->want_stamps) {
    if (!c->huge.ensure(16 + 8 * ym::HUGE_LIST)) return DEV_FAIL();
    hipMemsetAsync(c->huge.p, 0, 16, c->s);
    ym::launch_ls_list_diff(d_upd_off, b.pre_status, n, c->ls_min_diff, c->huge.as<uint32_t>(), c->s);
    hipMemcpyAsync(c->h_pinned + 9, c->huge.p, 4, hipMemcpyDeviceToHost, c->s);
    if (hipError_t e = hipStreamSynchronize(c->s); e != hipSuccess) return dev_err("long-document listing", e);
    if ((uint32_t)c->h_pinned[9]) {
      constexpr uint64_t OVW = 4u << 20; // overflow words for the parsed records
      constexpr size_t LSL = 4 + ym::LS_EW * ym::LS_LIST;
      const ym::LpArgs *lp = lp_args(c, LP_PMAX, b.v1x);
      if (lp && c->rec.ensure(nn * ym::REC_WORDS * 4) && c->ls_ovf.ensure(OVW * 4) && c->ls_list.ensure(LSL * 4) &&
          c->ls_done.ensure(nn)) {
        ym::LpArgs a = *lp;
        a.bytes = d_bytes;
        a.upd_off = d_upd_off;
        a.rec = c->rec.as<uint32_t>();
        a.ovf = c->ls_ovf.as<uint32_t>();
        a.huge = c->huge.as<uint32_t>();
        a.huge_base = 0;
        a.huge_cap = OVW;
        ym::launch_long_decode(a, c->s);
        hipMemsetAsync(c->ls_list.p, 0, 16, c->s);
        ym::launch_ls_collect(a, c->ls_list.as<uint32_t>(), c->s);
        hipMemcpyAsync(c->h_pinned + 256, c->ls_list.p, LSL * 4, hipMemcpyDeviceToHost, c->s);
        if (hipError_t e = hipStreamSynchronize(c->s); e != hipSuccess) return dev_err("long-document parse", e);
        ls = ls_entries((const uint32_t *)(c->h_pinned + 256));
        uint64_t words = 0;
        for (const LsEntry &e : ls) {
          ls_off.push_back(words);
          words += ls_scratch_words(e);
        }
        if (!ls.empty() && c->ls_scr.ensure(words * 4 + 64)) {
          hipMemsetAsync(c->ls_done.p, 0, nn, c->s);
          b.ls_done = c->ls_done.as<uint8_t>();
        } else {
          ls.clear();
        }
      }
      (void)hipGetLastError(); // a failed optional allocation leaves these documents to the planners
    }
  }
  auto ls_args = [&](size_t k) {
    ym::LsArgs a{};
    a.bytes = d_bytes;
    a.upd_off = d_upd_off;
    a.ov = c->ls_ovf.as<uint32_t>() + ls[k].ovf;
    a.mode = diff ? 1 : 2;
    a.v1x = b.v1x;
    a.frame = frame;
    a.sv = b.sv;
    a.sv_off = b.sv_off;
    a.sv_end = b.sv_end;
    a.out = c->arena.as<uint8_t>();
    a.size = ps.size;
    a.status = ps.status;
    a.path = ps.big;
    a.done = c->ls_done.as<uint8_t>();
    a.pack_off = c->pack_off.as<uint64_t>();
    ls_bind(a, ls[k], c->ls_scr.as<uint32_t>() + ls_off[k]);
    return a;
  };
  for (size_t k = 0; k < ls.size(); k++) ym::launch_ls_doc(ls_args(k), 0, c->s);
  ym::launch_plan(diff, 0, b, ps, c->s);
  if (hipGetLastError() != hipSuccess) return dev_err("plan launch");
  hipEventRecord(c->ev[1], c->s);
  hipMemcpyAsync(c->h_pinned + 9, c->counter.p, 4, hipMemcpyDeviceToHost, c->s);
  if (hipError_t e = hipStreamSynchronize(c->s); e != hipSuccess) return dev_err("plan", e);
  const uint32_t n_big = (uint32_t)(c->h_pinned[9] & 0xFFFFFFFFu);
  if (n_big) {
    ym::launch_big_need(d_upd_off, ps.big, n, c->need.as<uint64_t>(), c->s);
    ym::launch_scan_u64(c->need.as<uint64_t>(), c->spill_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
    uint64_t words = 0;
    if (!read_words(c, c->spill_off.as<uint64_t>() + n, 8, &words)) return DEV_FAIL();
    if (!c->plan_big.ensure(words * 4 + 64)) return DEV_FAIL();
    ps.bigscr = c->plan_big.as<uint32_t>();
    ym::launch_plan(diff, 1, b, ps, c->s);
  }
  hipEventRecord(c->ev[2], c->s);
  ym::launch_scan_u64(ps.size, c->pack_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
  uint64_t total = 0;
  if (!read_words(c, c->pack_off.as<uint64_t>() + n, 8, &total)) return DEV_FAIL();
  if (!c->arena.ensure(total + 64)) return DEV_FAIL();
  hipEventRecord(c->ev[4], c->s);
  ym::launch_exec(b, ps, c->pack_off.as<uint64_t>(), c->arena.as<uint8_t>(), c->s);
  for (size_t k = 0; k < ls.size(); k++) ym::launch_ls_doc(ls_args(k), 1, c->s);
  hipEventRecord(c->ev[3], c->s);
  if (hipError_t e = hipStreamSynchronize(c->s); e != hipSuccess) return dev_err("exec", e);
  if (hipGetLastError() != hipSuccess) return DEV_FAIL();
  float t01 = 0, t12 = 0, t43 = 0, t03 = 0;
  hipEventElapsedTime(&t01, c->ev[0], c->ev[1]);
  hipEventElapsedTime(&t12, c->ev[1], c->ev[2]);
  hipEventElapsedTime(&t43, c->ev[4], c->ev[3]);
  hipEventElapsedTime(&t03, c->ev[0], c->ev[3]);
  c->stats = ymerge_stats{};
  c->stats.n_docs = n_docs;
  c->stats.bytes_out = total;
  c->stats.docs_exact = n_big; // documents re-planned with length-sized scratch
  c->stats.docs_fast = n_docs - n_big;
  c->stats.ms_fast = t01;  // plan kernel (small pass)
  c->stats.ms_exact = t12; // big re-plan pass (incl. its scan)
  c->stats.ms_tail = t43;  // execute kernel
  c->stats.ms_total = t03;
  res->d_out = c->arena.as<uint8_t>();
  res->d_out_start = c->pack_off.as<uint64_t>();
  res->d_out_len = ps.size;
  res->d_status = ps.status;
  res->arena_bytes = c->arena.cap;
  res->out_bytes = total;
  return 0;
}

extern "C" int ysync_step1_v1_batch_device(ymerge_ctx *c, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                                           uint64_t n_docs, ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return plan_exec(c, false, d_bytes, d_upd_off, nullptr, nullptr, n_docs, res, 2);
}
extern "C" int ysync_step2_v1_batch_device(ymerge_ctx *c, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                                           const uint8_t *d_msg, const uint64_t *d_msg_off, uint64_t n_docs,
                                           ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return plan_exec(c, true, d_bytes, d_upd_off, d_msg, d_msg_off, n_docs, res, 1);
}

extern "C" int yencode_state_vector_from_update_v1_batch_device(ymerge_ctx *c, const uint8_t *d_bytes,
                                                                const uint64_t *d_upd_off, uint64_t n_docs,
                                                                ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return plan_exec(c, false, d_bytes, d_upd_off, nullptr, nullptr, n_docs, res);
}
extern "C" int ydiff_updates_v1_batch_device(ymerge_ctx *c, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                                             const uint8_t *d_sv, const uint64_t *d_sv_off, uint64_t n_docs,
                                             ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return plan_exec(c, true, d_bytes, d_upd_off, d_sv, d_sv_off, n_docs, res);
}

// ---------------------------------------------------------------- store-based compaction
// Each document's updates applied in order to a fresh yrs Doc (GC on), one transaction each,
// then encode_state_as_update_v1 (ycompact.hip).  Output slots as for the merge; packed
// offsets by a scan of the lengths.
static int compact_device(ymerge_ctx *c, const uint8_t *d_bytes, uint64_t n_bytes, const uint64_t *d_upd_off,
                          uint64_t n_updates, const uint64_t *d_doc_upd, uint64_t n_docs, ymerge_device_result *res) {
  resolve_times(c);
  if (hipSetDevice(c->device) != hipSuccess) return DEV_FAIL();
  if (n_docs > 0xFFFFFFFFull) return YMERGE_ERR_OTHER;
  const uint32_t n = (uint32_t)n_docs;
  const size_t nn = (size_t)n + 1;
  const uint64_t slots = 2 * n_bytes + 64 * (uint64_t)n_docs;
  if (!c->status.ensure(nn) || !c->path.ensure(nn) || !c->out_start.ensure(nn * 8) || !c->out_len.ensure(nn * 8) ||
      !c->pack_off.ensure(nn * 8) || !c->scan_tmp.ensure(ym::scan_tmp_elems(n) * 8 + 64) ||
      !ensure_keep(c, c->arena, slots + 4096, 0) || !c->need.ensure(nn * 8) || !c->scr_off.ensure(nn * 8) ||
      !c->counts.ensure(nn * ym::COMPACT_HDR_WORDS * 4))
    return DEV_FAIL();
  ym::BatchIn b{d_bytes, d_upd_off, d_doc_upd, n, nullptr, nullptr};
  ym::FastOut fo{c->arena.as<uint8_t>(), c->out_start.as<uint64_t>(), c->out_len.as<uint64_t>(),
                 c->status.as<uint8_t>(), c->path.as<uint8_t>(), nullptr, nullptr, nullptr};
  if (c->want_stamps) { // diagnostic: per-document phase cycles (ycompact.hip)
    if (!c->stamps.ensure(nn * 16 * 8)) return DEV_FAIL();
    hipMemsetAsync(c->stamps.p, 0, nn * 16 * 8, c->s);
    fo.stamps = c->stamps.as<uint64_t>();
    c->stamps_docs = n_docs;
  }
  hipEventRecord(c->ev[0], c->s);
  // per-document scratch from the counts (blocks, ranges, clients), then the store pass
  ym::launch_compact_count(b, c->counts.as<uint32_t>(), c->need.as<uint64_t>(), c->s);
  ym::launch_scan_u64(c->need.as<uint64_t>(), c->scr_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
  uint64_t words = 0;
  if (!read_words(c, c->scr_off.as<uint64_t>() + n, 8, &words)) return DEV_FAIL();
  if (!c->cscr.ensure(words * 4 + 64)) return DEV_FAIL();
  hipEventRecord(c->ev[2], c->s);
  ym::launch_compact(b, fo, c->counts.as<uint32_t>(), c->scr_off.as<uint64_t>(), c->cscr.as<uint32_t>(),
                     c->compact_lpw, c->s);
  if (hipGetLastError() != hipSuccess) return DEV_FAIL();
  hipEventRecord(c->ev[1], c->s);
  ym::launch_scan_u64(c->out_len.as<uint64_t>(), c->pack_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
  c->pack_stale = false;
  uint64_t total = 0;
  if (!read_words(c, c->pack_off.as<uint64_t>() + n, 8, &total)) return DEV_FAIL();
  float t01 = 0, t21 = 0;
  hipEventElapsedTime(&t01, c->ev[0], c->ev[1]);
  hipEventElapsedTime(&t21, c->ev[2], c->ev[1]);
  c->stats = ymerge_stats{};
  c->stats.n_docs = n_docs;
  c->stats.bytes_in = n_bytes;
  c->stats.bytes_out = total;
  c->stats.ms_total = t01;     // counts + scan + store pass
  c->stats.ms_exact = t21;     // k_compact
  c->stats.ms_decode = t01 - t21;
  res->d_out = c->arena.as<uint8_t>();
  res->d_out_start = c->out_start.as<uint64_t>();
  res->d_out_len = c->out_len.as<uint64_t>();
  res->d_status = c->status.as<uint8_t>();
  res->arena_bytes = c->arena.cap;
  res->out_bytes = total;
  return 0;
}
extern "C" int ycompact_updates_v1_batch_device(ymerge_ctx *c, const uint8_t *d_bytes, uint64_t n_bytes,
                                                const uint64_t *d_upd_off, uint64_t n_updates,
                                                const uint64_t *d_doc_upd, uint64_t n_docs, ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return compact_device(c, d_bytes, n_bytes, d_upd_off, n_updates, d_doc_upd, n_docs, res);
}

// ---------------------------------------------------------------- lib0 v2 (yv2.hip)
// v2 updates -> v1x arena (c->v2x, offsets c->v2x_off[n_upd + 1], status c->v2_ust)
static int v2_transcode(ymerge_ctx *c, const uint8_t *d_bytes, const uint64_t *d_upd_off, uint64_t n_upd,
                        uint64_t *total, uint64_t n_bytes = 0) {
  if (n_upd > 0xFFFFFFFFull) return YMERGE_ERR_OTHER;
  const size_t nn = (size_t)n_upd + 1;
  if (!c->v2x_sz.ensure(nn * 8) || !c->v2x_off.ensure(nn * 8) || !c->v2_ust.ensure(nn) ||
      !c->scan_tmp.ensure(ym::scan_tmp_elems((uint32_t)n_upd) * 8 + 64))
    return DEV_FAIL();
  // one walk into per-update scratch slots, then a packing copy (n_bytes known: the merge
  // entry; an overflowing slot falls back to the two walks below)
  if (n_bytes && c->v2_onepass && c->v2_over.ensure(64) && c->v2_scr.ensure(4 * n_bytes + 64 * nn + 64)) {
    hipMemsetAsync(c->v2_over.p, 0, 4, c->s);
    ym::launch_v2_decode_one(d_bytes, d_upd_off, n_upd, c->v2_scr.as<uint8_t>(), c->v2x_sz.as<uint64_t>(),
                             c->v2_ust.as<uint8_t>(), c->v2_over.as<uint32_t>(), c->s);
    ym::launch_scan_u64(c->v2x_sz.as<uint64_t>(), c->v2x_off.as<uint64_t>(), (uint32_t)n_upd,
                        c->scan_tmp.as<uint64_t>(), c->s);
    if (hipMemcpyAsync(c->h_pinned, c->v2x_off.as<uint64_t>() + n_upd, 8, hipMemcpyDeviceToHost, c->s) != hipSuccess ||
        hipMemcpyAsync(c->h_pinned + 1, c->v2_over.p, 4, hipMemcpyDeviceToHost, c->s) != hipSuccess ||
        hipStreamSynchronize(c->s) != hipSuccess)
      return DEV_FAIL();
    if ((c->h_pinned[1] & 0xFFFFFFFFu) == 0) {
      *total = c->h_pinned[0];
      if (!c->v2x.ensure(*total + 64)) return DEV_FAIL();
      ym::launch_v2_xpack(d_upd_off, n_upd, c->v2_scr.as<uint8_t>(), c->v2x_off.as<uint64_t>(), c->v2x.as<uint8_t>(),
                          c->s);
      return hipGetLastError() == hipSuccess ? 0 : DEV_FAIL();
    }
  }
  (void)hipGetLastError();
  ym::launch_v2_decode(false, d_bytes, d_upd_off, n_upd, c->v2x_sz.as<uint64_t>(), nullptr, c->v2_ust.as<uint8_t>(),
                       c->s);
  ym::launch_scan_u64(c->v2x_sz.as<uint64_t>(), c->v2x_off.as<uint64_t>(), (uint32_t)n_upd,
                      c->scan_tmp.as<uint64_t>(), c->s);
  if (!read_words(c, c->v2x_off.as<uint64_t>() + n_upd, 8, total)) return DEV_FAIL();
  if (!c->v2x.ensure(*total + 64)) return DEV_FAIL();
  ym::launch_v2_decode(true, d_bytes, d_upd_off, n_upd, c->v2x_off.as<uint64_t>(), c->v2x.as<uint8_t>(),
                       c->v2_ust.as<uint8_t>(), c->s);
  return hipGetLastError() == hipSuccess ? 0 : DEV_FAIL();
}
// v1x result -> v2 (mode 0 update, 1 state vector) in c->v2_out; `res` then describes it
static int v2_encode(ymerge_ctx *c, ymerge_device_result *res, uint32_t n, int mode) {
  const size_t nn = (size_t)n + 1;
  if (!c->v2_osz.ensure(nn * 8) || !c->v2_ooff.ensure(nn * 8) || !c->pack_off.ensure(nn * 8) ||
      !c->scan_tmp.ensure(ym::scan_tmp_elems(n) * 8 + 64))
    return DEV_FAIL();
  // full updates: one walk into per-document column streams, then k_v2_pack (state vectors:
  // the two walks, which only copy)
  const uint64_t scr_bytes = 2 * 11 * res->out_bytes + 64ull * 11 * n + 64;
  const bool one = mode == 0 && c->v2_onepass && c->need.ensure(nn * 8) && c->scr_off.ensure(nn * 8) &&
                   c->v2_colsz.ensure(nn * 11 * 4) && c->v2_over.ensure(64) && c->v2_scr.ensure(scr_bytes);
  (void)hipGetLastError(); // (a failed optional allocation: the two walks)
  uint64_t total = 0, over = 0;
  if (one) {
    hipMemsetAsync(c->v2_over.p, 0, 4, c->s);
    ym::launch_v2_encode_one(res->d_out, res->d_out_start, res->d_out_len, res->d_status, n, c->need.as<uint64_t>(),
                             c->scr_off.as<uint64_t>(), c->scan_tmp.as<uint64_t>(), c->v2_scr.as<uint8_t>(),
                             c->v2_colsz.as<uint32_t>(), c->v2_osz.as<uint64_t>(), c->v2_over.as<uint32_t>(), c->s);
  } else {
    ym::launch_v2_encode(false, res->d_out, res->d_out_start, res->d_out_len, res->d_status, n,
                         c->v2_osz.as<uint64_t>(), nullptr, mode, c->s);
  }
  ym::launch_scan_u64(c->v2_osz.as<uint64_t>(), c->v2_ooff.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
  if (hipMemcpyAsync(c->h_pinned, c->v2_ooff.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, c->s) != hipSuccess ||
      (one && hipMemcpyAsync(c->h_pinned + 1, c->v2_over.p, 4, hipMemcpyDeviceToHost, c->s) != hipSuccess) ||
      hipStreamSynchronize(c->s) != hipSuccess)
    return DEV_FAIL();
  total = c->h_pinned[0];
  over = one ? (c->h_pinned[1] & 0xFFFFFFFFu) : 1;
  if (!c->v2_out.ensure(total + 64)) return DEV_FAIL();
  if (one && !over)
    ym::launch_v2_pack(res->d_out_len, res->d_status, n, c->scr_off.as<uint64_t>(), c->v2_scr.as<uint8_t>(),
                       c->v2_colsz.as<uint32_t>(), c->v2_ooff.as<uint64_t>(), c->v2_out.as<uint8_t>(), c->s);
  else
    ym::launch_v2_encode(true, res->d_out, res->d_out_start, res->d_out_len, res->d_status, n,
                         c->v2_ooff.as<uint64_t>(), c->v2_out.as<uint8_t>(), mode, c->s);
  // packed offsets of the result (pack_to_host copies the arena in their order)
  c->pack_stale = false;
  if (hipMemcpyAsync(c->pack_off.p, c->v2_ooff.p, nn * 8, hipMemcpyDeviceToDevice, c->s) != hipSuccess)
    return DEV_FAIL();
  if (hipStreamSynchronize(c->s) != hipSuccess || hipGetLastError() != hipSuccess) return DEV_FAIL();
  res->d_out = c->v2_out.as<uint8_t>();
  res->d_out_start = c->v2_ooff.as<uint64_t>();
  res->d_out_len = c->v2_osz.as<uint64_t>();
  res->arena_bytes = c->v2_out.cap;
  res->out_bytes = total;
  return 0;
}
static int merge_v2_device(ymerge_ctx *c, const uint8_t *d_bytes, uint64_t n_bytes, const uint64_t *d_upd_off,
                           uint64_t n_updates, const uint64_t *d_doc_upd, uint64_t n_docs, ymerge_device_result *res) {
  if (hipSetDevice(c->device) != hipSuccess) return DEV_FAIL();
  if (n_docs > 0xFFFFFFFFull) return YMERGE_ERR_OTHER;
  uint64_t xbytes = 0;
  hipEventRecord(c->v2ev[0], c->s);
  int st = v2_transcode(c, d_bytes, d_upd_off, n_updates, &xbytes, n_bytes);
  if (st) return st;
  hipEventRecord(c->v2ev[1], c->s);
  st = merge_device(c, c->v2x.as<uint8_t>(), xbytes, c->v2x_off.as<uint64_t>(), n_updates, d_doc_upd, n_docs, res);
  if (st) return st;
  hipEventRecord(c->v2ev[2], c->s);
  ym::launch_v2_doc_status(d_doc_upd, c->v2_ust.as<uint8_t>(), (uint32_t)n_docs, res->d_status,
                           (uint64_t *)res->d_out_len, c->s);
  st = v2_encode(c, res, (uint32_t)n_docs, 0);
  hipEventRecord(c->v2ev[3], c->s);
  hipEventSynchronize(c->v2ev[3]);
  c->stats.bytes_in = n_bytes;
  c->stats.bytes_out = res->out_bytes;
  hipEventElapsedTime(&c->stats.ms_v2_decode, c->v2ev[0], c->v2ev[1]);
  hipEventElapsedTime(&c->stats.ms_v2_merge, c->v2ev[1], c->v2ev[2]);
  hipEventElapsedTime(&c->stats.ms_v2_encode, c->v2ev[2], c->v2ev[3]);
  return st;
}
// diff_updates_v2 (diff = true) / encode_state_vector_from_update_v2: one update per document
static int plan_v2_device(ymerge_ctx *c, bool diff, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                          const uint8_t *d_sv, const uint64_t *d_sv_off, uint64_t n_docs, ymerge_device_result *res) {
  if (hipSetDevice(c->device) != hipSuccess) return DEV_FAIL();
  if (n_docs > 0xFFFFFFFFull) return YMERGE_ERR_OTHER;
  const uint32_t n = (uint32_t)n_docs;
  uint64_t xbytes = 0;
  int st = v2_transcode(c, d_bytes, d_upd_off, n_docs, &xbytes);
  if (st) return st;
  if (!c->v2_svoff.ensure((n + 1) * 8) || !c->v2_svend.ensure((n + 1) * 8) || !c->v2_pre.ensure(n + 1))
    return DEV_FAIL();
  ym::launch_v2_sv_parse(diff ? d_sv : nullptr, d_sv_off, c->v2_ust.as<uint8_t>(), n, c->v2_svoff.as<uint64_t>(),
                         c->v2_svend.as<uint64_t>(), c->v2_pre.as<uint8_t>(), c->s);
  st = plan_exec(c, diff, c->v2x.as<uint8_t>(), c->v2x_off.as<uint64_t>(), d_sv,
                 diff ? c->v2_svoff.as<uint64_t>() : nullptr, n_docs, res, 0,
                 diff ? c->v2_svend.as<uint64_t>() : nullptr, c->v2_pre.as<uint8_t>());
  if (st) return st;
  return v2_encode(c, res, n, diff ? 0 : 1);
}

// lib0 v1 -> v2 for every update of an arena (Update::decode_v1(u).encode_v2(), yrs/src/
// update.rs:714-749 + updates/encoder.rs): each update merged alone (a one-update document)
// and written by the v2 encoder.  Used to feed the lib0 v2 paths (bench, tests).
extern "C" int yconvert_updates_v1_to_v2_batch_device(ymerge_ctx *c, const uint8_t *d_bytes, uint64_t n_bytes,
                                                     const uint64_t *d_upd_off, uint64_t n_updates,
                                                     ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return DEV_FAIL();
  if (n_updates > 0xFFFFFFFFull) return YMERGE_ERR_OTHER;
  std::vector<uint64_t> iota(n_updates + 1);
  for (uint64_t i = 0; i <= n_updates; i++) iota[i] = i;
  if (!c->in_doc_upd.ensure((n_updates + 1) * 8) ||
      hipMemcpyAsync(c->in_doc_upd.p, iota.data(), (n_updates + 1) * 8, hipMemcpyHostToDevice, c->s) != hipSuccess)
    return DEV_FAIL();
  int st = merge_device(c, d_bytes, n_bytes, d_upd_off, n_updates, c->in_doc_upd.as<uint64_t>(), n_updates, res);
  if (st) return st;
  return v2_encode(c, res, (uint32_t)n_updates, 0);
}

extern "C" int ymerge_updates_v2_batch_device(ymerge_ctx *c, const uint8_t *d_bytes, uint64_t n_bytes,
                                              const uint64_t *d_upd_off, uint64_t n_updates, const uint64_t *d_doc_upd,
                                              uint64_t n_docs, ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return merge_v2_device(c, d_bytes, n_bytes, d_upd_off, n_updates, d_doc_upd, n_docs, res);
}
extern "C" int ydiff_updates_v2_batch_device(ymerge_ctx *c, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                                             const uint8_t *d_sv, const uint64_t *d_sv_off, uint64_t n_docs,
                                             ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return plan_v2_device(c, true, d_bytes, d_upd_off, d_sv, d_sv_off, n_docs, res);
}
extern "C" int yencode_state_vector_from_update_v2_batch_device(ymerge_ctx *c, const uint8_t *d_bytes,
                                                                const uint64_t *d_upd_off, uint64_t n_docs,
                                                                ymerge_device_result *res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  return plan_v2_device(c, false, d_bytes, d_upd_off, nullptr, nullptr, n_docs, res);
}

static int pack_to_host(ymerge_ctx *c, const ymerge_device_result *res, uint64_t n_docs, uint8_t *out,
                        uint64_t *out_off, uint8_t *status) {
  const uint32_t n = (uint32_t)n_docs;
  if (!c->packed.ensure(res->out_bytes + 64)) return DEV_FAIL();
  if (c->pack_stale) { // packed offsets of a merge whose documents were all written by k_lean
    ym::launch_scan_u64(res->d_out_len, c->pack_off.as<uint64_t>(), n, c->scan_tmp.as<uint64_t>(), c->s);
    c->pack_stale = false;
  }
  ym::launch_pack(res->d_out, res->d_out_start, res->d_out_len, c->pack_off.as<uint64_t>(),
                  c->packed.as<uint8_t>(), n, c->s);
  if (out && res->out_bytes && !copy_d2h(c, out, c->packed.p, res->out_bytes)) return DEV_FAIL();
  if (out_off && hipMemcpyAsync(out_off, c->pack_off.p, (n_docs + 1) * 8, hipMemcpyDeviceToHost, c->s) != hipSuccess)
    return DEV_FAIL();
  if (status && n_docs && hipMemcpyAsync(status, res->d_status, n_docs, hipMemcpyDeviceToHost, c->s) != hipSuccess)
    return DEV_FAIL();
  return hipStreamSynchronize(c->s) == hipSuccess ? 0 : DEV_FAIL();
}

extern "C" int ymerge_result_to_host(ymerge_ctx *c, const ymerge_device_result *res, uint64_t n_docs, uint8_t *out,
                                     uint64_t *out_off, uint8_t *status) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  return pack_to_host(c, res, n_docs, out, out_off, status);
}

// diagnostic: copy per-document phase stamps (16 x u64 per document) of the last batch
extern "C" int ymerge_debug_stamps(ymerge_ctx *c, uint64_t n_docs, uint64_t *dst) {
  if (!c || !dst) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->want_stamps || !c->stamps.p) return YMERGE_ERR_OTHER;
  if (n_docs > c->stamps_docs) n_docs = c->stamps_docs; // never past the last batch's stamps
  if (!n_docs) return 0;
  hipSetDevice(c->device);
  if (hipMemcpy(dst, c->stamps.p, n_docs * 16 * 8, hipMemcpyDeviceToHost) != hipSuccess) return DEV_FAIL();
  return 0;
}

extern "C" void ymerge_ctx_set_stage_timing(ymerge_ctx *c, int on) {
  if (!c) return;
  std::lock_guard<std::mutex> g(c->mu);
  c->timing = on != 0;
}

extern "C" void ymerge_last_stats(ymerge_ctx *c, ymerge_stats *st) {
  if (!c || !st) return;
  std::lock_guard<std::mutex> g(c->mu);
  resolve_times(c);
  *st = c->stats;
}

static int host_merge(ymerge_ctx *c, int version, const uint8_t *bytes, const uint64_t *upd_off,
                      uint64_t n_updates, const uint64_t *doc_upd, uint64_t n_docs, ymerge_batch_result **out);
extern "C" int ymerge_updates_v1_batch(ymerge_ctx *c, const uint8_t *bytes, const uint64_t *upd_off,
                                       uint64_t n_updates, const uint64_t *doc_upd, uint64_t n_docs,
                                       ymerge_batch_result **out) {
  return host_merge(c, 1, bytes, upd_off, n_updates, doc_upd, n_docs, out);
}
extern "C" int ycompact_updates_v1_batch(ymerge_ctx *c, const uint8_t *bytes, const uint64_t *upd_off,
                                         uint64_t n_updates, const uint64_t *doc_upd, uint64_t n_docs,
                                         ymerge_batch_result **out) {
  return host_merge(c, 3, bytes, upd_off, n_updates, doc_upd, n_docs, out);
}
extern "C" int ymerge_updates_v2_batch(ymerge_ctx *c, const uint8_t *bytes, const uint64_t *upd_off,
                                       uint64_t n_updates, const uint64_t *doc_upd, uint64_t n_docs,
                                       ymerge_batch_result **out) {
  return host_merge(c, 2, bytes, upd_off, n_updates, doc_upd, n_docs, out);
}
// Large host batches are pipelined over groups of documents (~48 MB of input each): a
// producer thread stages group g + 1 into HBM (stream s_in) while this thread merges group g
// on the engine stream and the DMA engine returns group g - 1's packed output (stream
// s_out) straight into the pinned result arena.  H2D, compute and D2H overlap; each
// group is an ordinary merge_device call over its documents and its slice of the input
// arena (offsets rebased to the slice), so device memory scales with the group.
constexpr uint64_t GROUP_BYTES = 48ull << 20;
static int host_merge_pipelined(ymerge_ctx *c, const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_updates,
                                const uint64_t *doc_upd, uint64_t n_docs, ymerge_batch_result **out) {
  const uint64_t nbytes = upd_off[n_updates];
  // groups of whole documents
  std::vector<uint64_t> gd = {0};
  for (uint64_t d = 0; d < n_docs; d++)
    if (upd_off[doc_upd[d + 1]] - upd_off[doc_upd[gd.back()]] >= GROUP_BYTES && gd.size() < 64) gd.push_back(d + 1);
  if (gd.back() != n_docs) gd.push_back(n_docs);
  const size_t G = gd.size() - 1;
  if (!c->s_in && hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking) != hipSuccess) return DEV_FAIL();
  if (!c->s_out && hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking) != hipSuccess) return DEV_FAIL();
  for (size_t k = 0; k < G; k++)
    if (!c->ev_in[k] && hipEventCreateWithFlags(&c->ev_in[k], hipEventDisableTiming) != hipSuccess)
      return DEV_FAIL();
  for (int k = 0; k < 2; k++)
    if ((!c->ev_out[k] && hipEventCreateWithFlags(&c->ev_out[k], hipEventDisableTiming) != hipSuccess) ||
        (!c->ev_packed[k] && hipEventCreateWithFlags(&c->ev_packed[k], hipEventDisableTiming) != hipSuccess))
      return DEV_FAIL();
  if (!stage_init(c) || !c->in_bytes.ensure(nbytes + 16) || !c->in_upd_off.ensure((n_updates + G + 1) * 8) ||
      !c->grp_doc_upd.ensure((n_docs + G + 1) * 8))
    return DEV_FAIL();
  // rebased tables of every group: its documents index its slice of the update offsets, and
  // those count from the group's first byte rounded down to 16 (the kernels' aligned loads), so
  // each merge_device call sizes its slots and scratch by the group, not the whole batch.  The
  // producer stages each group's slices of the caller's tables with its bytes and rebases them
  // on the device (k_rebase_u64): rebasing on the host and uploading the tables up front
  // (8 B per update, C2: 80 MB) serialised ~25 ms before the first H2D (round 4-5: C-ABI
  // entry 31 -> 8 GB/s on C2).
  std::vector<uint64_t> gdu_off(G + 1, 0), guo_off(G + 1, 0), gbase(G);
  for (size_t k = 0; k < G; k++) {
    gdu_off[k + 1] = gdu_off[k] + (gd[k + 1] - gd[k]) + 1;
    const uint64_t u0 = doc_upd[gd[k]], u1 = doc_upd[gd[k + 1]];
    gbase[k] = upd_off[u0] & ~15ull;
    guo_off[k + 1] = guo_off[k] + (u1 - u0) + 1;
  }
  static const bool trace = getenv("YMERGE_HOST_TRACE") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  // producer: stage every group's tables and bytes through the pinned ring on s_in, one event per group
  std::atomic<int> prod_rc{0};
  std::atomic<size_t> recorded{0}; // groups whose ev_in the producer has recorded
  std::thread producer([&] {
    hipSetDevice(c->device);
    // pieces packed into whole 32 MB pinned chunks (a group's tables and bytes share chunks;
    // a half-empty chunk per piece left the DMA idle between pieces), flushed at group ends
    size_t i = 0, fill = 0; // chunks issued, bytes in the current one
    struct Piece {
      uint8_t *dst;
      size_t at, n;
    };
    std::vector<Piece> pieces;
    auto flush = [&]() -> bool {
      if (!fill) return true;
      const int b = (int)(i & 1);
      for (const Piece &q : pieces)
        if (hipMemcpyAsync(q.dst, c->stage[b] + q.at, q.n, hipMemcpyHostToDevice, c->s_in) != hipSuccess) return false;
      if (hipEventRecord(c->stage_ev[b], c->s_in) != hipSuccess) return false;
      pieces.clear();
      fill = 0;
      i++;
      // the next chunk's buffer must have drained (its DMA was issued two chunks ago)
      return i < 2 || hipEventSynchronize(c->stage_ev[i & 1]) == hipSuccess;
    };
    auto add = [&](uint8_t *dst, const uint8_t *src, uint64_t n) -> bool {
      while (n) {
        const size_t take = std::min<uint64_t>(STAGE_CHUNK - fill, n);
        par_memcpy(c->stage[i & 1] + fill, src, take);
        pieces.push_back({dst, fill, take});
        fill += take;
        dst += take;
        src += take;
        n -= take;
        if (fill == STAGE_CHUNK && !flush()) return false;
      }
      return true;
    };
    for (size_t k = 0; k < G && !prod_rc; k++) {
      const uint64_t d0 = gd[k], nd = gd[k + 1] - gd[k], u0 = doc_upd[d0], nu = doc_upd[gd[k + 1]] - u0;
      uint64_t *guo = c->in_upd_off.as<uint64_t>() + guo_off[k], *gdu = c->grp_doc_upd.as<uint64_t>() + gdu_off[k];
      const uint64_t a = upd_off[u0], z = upd_off[u0 + nu];
      if (!add((uint8_t *)guo, (const uint8_t *)(upd_off + u0), (nu + 1) * 8) ||
          !add((uint8_t *)gdu, (const uint8_t *)(doc_upd + d0), (nd + 1) * 8) ||
          !add(c->in_bytes.as<uint8_t>() + a, bytes + a, z - a) || !flush()) {
        prod_rc = DEV_FAIL();
        break;
      }
      ym::launch_rebase_u64(guo, nu + 1, gbase[k], c->s_in);
      ym::launch_rebase_u64(gdu, nd + 1, u0, c->s_in);
      if (hipEventRecord(c->ev_in[k], c->s_in) != hipSuccess) {
        prod_rc = DEV_FAIL();
        break;
      }
      if (trace) fprintf(stderr, "ymerge host: group %zu staged at %.2f ms\n", k, ms());
      recorded.store(k + 1);
    }
  });
  // result arena: the merge output of a document fits its slot (2 x its bytes + 64)
  ymerge_batch_result *r = alloc_result(n_docs, 2 * nbytes + 64 * n_docs);
  int rc = r ? 0 : YMERGE_ERR_NOT_ENOUGH_MEMORY;
  uint64_t obase = 0;
  for (size_t k = 0; k < G && !rc; k++) {
    const uint64_t nd = gd[k + 1] - gd[k];
    // order the engine stream after group k's H2D: wait (host) until the producer has
    // recorded its event (waiting on an event not yet recorded would not wait at all)
    for (;;) {
      if (prod_rc) {
        rc = prod_rc;
        break;
      }
      if (recorded.load() > k) break;
      std::this_thread::yield();
    }
    if (rc || hipStreamWaitEvent(c->s, c->ev_in[k], 0) != hipSuccess) {
      rc = rc ? rc : DEV_FAIL();
      break;
    }
    ymerge_device_result dr{};
    const uint64_t u0 = doc_upd[gd[k]], u1 = doc_upd[gd[k + 1]];
    rc = merge_device(c, c->in_bytes.as<uint8_t>() + gbase[k], upd_off[u1] - gbase[k],
                      c->in_upd_off.as<uint64_t>() + guo_off[k], u1 - u0, c->grp_doc_upd.as<uint64_t>() + gdu_off[k], nd,
                      &dr);
    if (rc) break;
    // pack group k into packed2[k & 1] once group k - 2's D2H from it has drained
    const int pb = (int)(k & 1);
    if (k >= 2 && hipStreamWaitEvent(c->s, c->ev_out[pb], 0) != hipSuccess) {
      rc = YMERGE_ERR_DEVICE;
      break;
    }
    if (!c->packed2[pb].ensure(dr.out_bytes + 64)) {
      rc = YMERGE_ERR_DEVICE;
      break;
    }
    if (c->pack_stale) {
      ym::launch_scan_u64(dr.d_out_len, c->pack_off.as<uint64_t>(), (uint32_t)nd, c->scan_tmp.as<uint64_t>(), c->s);
      c->pack_stale = false;
    }
    ym::launch_pack(dr.d_out, dr.d_out_start, dr.d_out_len, c->pack_off.as<uint64_t>(), c->packed2[pb].as<uint8_t>(),
                    (uint32_t)nd, c->s);
    // offsets and statuses (small) now; the bytes on s_out behind the pack
    if (hipMemcpyAsync(r->out_off + gd[k], c->pack_off.p, (nd + 1) * 8, hipMemcpyDeviceToHost, c->s) != hipSuccess ||
        hipMemcpyAsync(r->status + gd[k], dr.d_status, nd, hipMemcpyDeviceToHost, c->s) != hipSuccess ||
        hipEventRecord(c->ev_packed[pb], c->s) != hipSuccess || hipStreamSynchronize(c->s) != hipSuccess) {
      rc = YMERGE_ERR_DEVICE;
      break;
    }
    for (uint64_t d = gd[k]; d <= gd[k + 1]; d++) r->out_off[d] += obase;
    if (hipStreamWaitEvent(c->s_out, c->ev_packed[pb], 0) != hipSuccess ||
        (dr.out_bytes && hipMemcpyAsync(r->out + obase, c->packed2[pb].p, dr.out_bytes, hipMemcpyDeviceToHost,
                                        c->s_out) != hipSuccess) ||
        hipEventRecord(c->ev_out[pb], c->s_out) != hipSuccess) {
      rc = YMERGE_ERR_DEVICE;
      break;
    }
    obase += dr.out_bytes;
    if (trace) fprintf(stderr, "ymerge host: group %zu merged + packed at %.2f ms\n", k, ms());
  }
  producer.join();
  if (!rc && prod_rc) rc = prod_rc;
  if (hipStreamSynchronize(c->s_out) != hipSuccess && !rc) rc = YMERGE_ERR_DEVICE;
  if (rc) {
    ymerge_batch_result_destroy(r);
    return rc;
  }
  r->out_bytes = obase;
  if (trace) fprintf(stderr, "ymerge host: %zu groups done at %.2f ms\n", G, ms());
  *out = r;
  return 0;
}

static int host_merge(ymerge_ctx *c, int version, const uint8_t *bytes, const uint64_t *upd_off,
                      uint64_t n_updates, const uint64_t *doc_upd, uint64_t n_docs, ymerge_batch_result **out) {
  if (!c || !out) return YMERGE_ERR_OTHER;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  uint64_t nbytes = upd_off[n_updates];
  if (version == 1 && nbytes >= 2 * GROUP_BYTES && n_docs >= 2 && !c->want_stamps)
    return host_merge_pipelined(c, bytes, upd_off, n_updates, doc_upd, n_docs, out);
  if (!c->in_bytes.ensure(nbytes + 16) || !c->in_upd_off.ensure((n_updates + 1) * 8) ||
      !c->in_doc_upd.ensure((n_docs + 1) * 8))
    return DEV_FAIL();
  if (!copy_h2d(c, c->in_bytes.p, bytes, nbytes)) return DEV_FAIL();
  if (hipMemcpyAsync(c->in_upd_off.p, upd_off, (n_updates + 1) * 8, hipMemcpyHostToDevice, c->s) != hipSuccess ||
      hipMemcpyAsync(c->in_doc_upd.p, doc_upd, (n_docs + 1) * 8, hipMemcpyHostToDevice, c->s) != hipSuccess)
    return DEV_FAIL();
  ymerge_device_result dr{};
  int st = (version == 3 ? compact_device : version == 2 ? merge_v2_device : merge_device)(c, c->in_bytes.as<uint8_t>(), nbytes,
                                                           c->in_upd_off.as<uint64_t>(), n_updates,
                                                           c->in_doc_upd.as<uint64_t>(), n_docs, &dr);
  if (st) return st;
  ymerge_batch_result *r = alloc_result(n_docs, dr.out_bytes);
  if (!r) return YMERGE_ERR_NOT_ENOUGH_MEMORY;
  st = pack_to_host(c, &dr, n_docs, r->out, r->out_off, r->status);
  if (st) {
    ymerge_batch_result_destroy(r);
    return st;
  }
  *out = r;
  return 0;
}

// Result arenas of the host entries come from a process-wide pool of pinned buffers: the
// D2H lands in them directly (no bounce copy), and a reused buffer has no first-touch page
// faults (a fresh 165 MB malloc arena costs ~20 ms of faults, its free ~18 ms of unmapping).
// Freed arenas stay pooled up to POOL_MAX bytes.
namespace {
struct ResultBox {
  ymerge_batch_result r; // first member: the public pointer is the box
  size_t out_cap;
  bool pinned;
};
std::mutex g_pool_mu;
std::multimap<size_t, uint8_t *> g_pool; // capacity -> pinned arena
size_t g_pool_bytes = 0;
constexpr size_t POOL_MAX = 4ull << 30;
uint8_t *pool_get(size_t n, size_t *cap, bool *pinned) {
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    auto it = g_pool.lower_bound(n);
    if (it != g_pool.end() && it->first <= 2 * n + (1u << 20)) {
      uint8_t *p = it->second;
      *cap = it->first;
      g_pool_bytes -= it->first;
      g_pool.erase(it);
      *pinned = true;
      return p;
    }
  }
  const size_t c = ((n + 1) + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
  uint8_t *p = nullptr;
  if (c >= (4u << 20) && hipHostMalloc((void **)&p, c, hipHostMallocDefault) == hipSuccess) {
    *cap = c;
    *pinned = true;
    return p;
  }
  (void)hipGetLastError();
  *cap = n + 1;
  *pinned = false;
  return (uint8_t *)malloc(n + 1);
}
void pool_put(uint8_t *p, size_t cap, bool pinned) {
  if (!p) return;
  if (!pinned) {
    free(p);
    return;
  }
  std::lock_guard<std::mutex> g(g_pool_mu);
  if (g_pool_bytes + cap <= POOL_MAX) {
    g_pool.emplace(cap, p);
    g_pool_bytes += cap;
  } else {
    hipHostFree(p);
  }
}
ymerge_batch_result *alloc_result(uint64_t n_docs, uint64_t out_bytes) {
  auto *b = (ResultBox *)calloc(1, sizeof(ResultBox));
  if (!b) return nullptr;
  ymerge_batch_result *r = &b->r;
  r->n_docs = n_docs;
  r->out_bytes = out_bytes;
  r->out = pool_get(out_bytes, &b->out_cap, &b->pinned);
  r->out_off = (uint64_t *)malloc((n_docs + 1) * 8);
  r->status = (uint8_t *)malloc(n_docs + 1);
  if (!r->out || !r->out_off || !r->status) {
    ymerge_batch_result_destroy(r);
    return nullptr;
  }
  return r;
}
} // namespace

extern "C" void ymerge_batch_result_destroy(ymerge_batch_result *r) {
  if (!r) return;
  auto *b = (ResultBox *)r;
  pool_put(r->out, b->out_cap, b->pinned);
  free(r->out_off);
  free(r->status);
  free(b);
}

// ---------------------------------------------------------------- multi-device (one node)
// Documents are independent (yrs/src/alt.rs:15-81 take one document's updates), so a batch
// spreads over the contexts' devices by document hash with no cross-device traffic: document
// d goes to context splitmix64(id) % n_ctx (id = doc_ids[d], else d: the partition bench.py
// uses across ranks, workloads.shard_ids).  Each shard's sub-batch is gathered from the
// caller's arena and run on its own host thread (one HIP stream per context); the outputs
// are put back in input order.
static uint64_t doc_hash(uint64_t id) {
  uint64_t z = id + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Shard {
  std::vector<uint64_t> docs;           // input document indices, ascending
  std::vector<uint8_t> bytes;           // gathered arena (+16 readable bytes)
  std::vector<uint64_t> upd_off, doc_upd, sv_off;
  std::vector<uint8_t> sv;
  ymerge_batch_result *res = nullptr;
  int rc = 0;
};

// op: 0 merge (doc_upd groups updates), 1 diff (one update + one state vector per document)
static int run_multi(ymerge_ctx *const *ctxs, uint32_t n_ctx, int op, const uint8_t *bytes, const uint64_t *upd_off,
                     const uint64_t *doc_upd, const uint8_t *sv, const uint64_t *sv_off, uint64_t n_docs,
                     const uint64_t *doc_ids, ymerge_batch_result **out) {
  if (!ctxs || !n_ctx || !out) return YMERGE_ERR_OTHER;
  for (uint32_t k = 0; k < n_ctx; k++)
    if (!ctxs[k]) return YMERGE_ERR_OTHER;
  std::vector<Shard> sh(n_ctx);
  std::vector<uint32_t> owner(n_docs);
  for (uint64_t d = 0; d < n_docs; d++) {
    const uint32_t k = (uint32_t)(doc_hash(doc_ids ? doc_ids[d] : d) % n_ctx);
    owner[d] = k;
    sh[k].docs.push_back(d);
  }
  auto work = [&](uint32_t k) {
    Shard &s = sh[k];
    const uint64_t n = s.docs.size();
    s.upd_off.push_back(0);
    if (op == 0) s.doc_upd.push_back(0);
    else s.sv_off.push_back(0);
    for (uint64_t d : s.docs) {
      const uint64_t u0 = op == 0 ? doc_upd[d] : d, u1 = op == 0 ? doc_upd[d + 1] : d + 1;
      const uint64_t base = s.bytes.size();
      s.bytes.insert(s.bytes.end(), bytes + upd_off[u0], bytes + upd_off[u1]);
      for (uint64_t u = u0; u < u1; u++) s.upd_off.push_back(base + upd_off[u + 1] - upd_off[u0]);
      if (op == 0) s.doc_upd.push_back(s.upd_off.size() - 1);
      else {
        s.sv.insert(s.sv.end(), sv + sv_off[d], sv + sv_off[d + 1]);
        s.sv_off.push_back(s.sv.size());
      }
    }
    s.bytes.resize(s.bytes.size() + 16, 0);
    if (op == 1) s.sv.resize(s.sv.size() + 16, 0);
    if (op == 0)
      s.rc = ymerge_updates_v1_batch(ctxs[k], s.bytes.data(), s.upd_off.data(), s.upd_off.size() - 1,
                                     s.doc_upd.data(), n, &s.res);
    else
      s.rc = ydiff_updates_v1_batch(ctxs[k], s.bytes.data(), s.upd_off.data(), s.sv.data(), s.sv_off.data(), n,
                                    &s.res);
  };
  std::vector<std::thread> th;
  for (uint32_t k = 1; k < n_ctx; k++) th.emplace_back(work, k);
  work(0);
  for (auto &t : th) t.join();
  int rc = 0;
  uint64_t total = 0;
  for (auto &s : sh) {
    if (s.rc && !rc) rc = s.rc;
    if (s.res) total += s.res->out_bytes;
  }
  ymerge_batch_result *r = rc ? nullptr : alloc_result(n_docs, total);
  if (!rc && !r) rc = YMERGE_ERR_NOT_ENOUGH_MEMORY;
  if (!rc) {
    std::vector<uint64_t> pos(n_ctx, 0);
    uint64_t o = 0;
    r->out_off[0] = 0;
    for (uint64_t d = 0; d < n_docs; d++) {
      const uint32_t k = owner[d];
      const ymerge_batch_result *sr = sh[k].res;
      const uint64_t i = pos[k]++;
      const uint64_t a = sr->out_off[i], len = sr->out_off[i + 1] - a;
      if (len) memcpy(r->out + o, sr->out + a, len);
      o += len;
      r->out_off[d + 1] = o;
      r->status[d] = sr->status[i];
    }
    *out = r;
  }
  for (auto &s : sh) ymerge_batch_result_destroy(s.res);
  return rc;
}

extern "C" int ymerge_updates_v1_batch_multi(ymerge_ctx *const *ctxs, uint32_t n_ctx, const uint8_t *bytes,
                                             const uint64_t *upd_off, uint64_t n_updates, const uint64_t *doc_upd,
                                             uint64_t n_docs, const uint64_t *doc_ids, ymerge_batch_result **res) {
  (void)n_updates;
  return run_multi(ctxs, n_ctx, 0, bytes, upd_off, doc_upd, nullptr, nullptr, n_docs, doc_ids, res);
}
extern "C" int ydiff_updates_v1_batch_multi(ymerge_ctx *const *ctxs, uint32_t n_ctx, const uint8_t *bytes,
                                            const uint64_t *upd_off, const uint8_t *sv, const uint64_t *sv_off,
                                            uint64_t n_docs, const uint64_t *doc_ids, ymerge_batch_result **res) {
  return run_multi(ctxs, n_ctx, 1, bytes, upd_off, nullptr, sv, sv_off, n_docs, doc_ids, res);
}

// ---------------------------------------------------------------- single document API
// The single-document calls run on one lazily created context per device; the device is
// ymerge_set_default_device(), else env YMERGE_DEVICE, else 0.
static std::mutex g_default_mu;
static std::vector<ymerge_ctx *> g_default;
static int g_default_device = -1;
extern "C" int ymerge_set_default_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return DEV_FAIL();
  std::lock_guard<std::mutex> g(g_default_mu);
  g_default_device = device;
  return 0;
}
static ymerge_ctx *default_ctx() {
  std::lock_guard<std::mutex> g(g_default_mu);
  if (g_default_device < 0) {
    const char *v = getenv("YMERGE_DEVICE");
    g_default_device = v ? atoi(v) : 0;
  }
  const int dev = g_default_device;
  if (dev < 0) return nullptr;
  if ((size_t)dev >= g_default.size()) g_default.resize(dev + 1, nullptr);
  if (!g_default[dev]) g_default[dev] = ymerge_ctx_create(dev);
  return g_default[dev];
}

extern "C" uint8_t ymerge_last_error(void) { return g_last_error; }
extern "C" const char *ymerge_last_error_message(void) { return g_last_msg; }

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
  if (!res) {
    g_last_error = YMERGE_ERR_NOT_ENOUGH_MEMORY;
    ymerge_batch_result_destroy(r);
    return nullptr;
  }
  memcpy(res, r->out + r->out_off[0], n);
  *out_len = (uint32_t)n;
  ymerge_batch_result_destroy(r);
  return res;
}

// host buffers of one (or more) documents -> device -> plan/exec -> host
static int host_plan_exec(ymerge_ctx *c, bool diff, const uint8_t *bytes, const uint64_t *upd_off,
                          const uint8_t *sv, const uint64_t *sv_off, uint64_t n_docs, ymerge_batch_result **out,
                          uint32_t frame = 0, int version = 1) {
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  const uint64_t nbytes = upd_off[n_docs], nsv = diff ? sv_off[n_docs] : 0;
  if (!c->in_bytes.ensure(nbytes + 16) || !c->in_upd_off.ensure((n_docs + 1) * 8) ||
      (diff && (!c->in_sv.ensure(nsv + 16) || !c->in_sv_off.ensure((n_docs + 1) * 8))))
    return DEV_FAIL();
  if (!copy_h2d(c, c->in_bytes.p, bytes, nbytes)) return DEV_FAIL();
  if (hipMemcpyAsync(c->in_upd_off.p, upd_off, (n_docs + 1) * 8, hipMemcpyHostToDevice, c->s) != hipSuccess)
    return DEV_FAIL();
  if (diff) {
    if (!copy_h2d(c, c->in_sv.p, sv, nsv)) return DEV_FAIL();
    if (hipMemcpyAsync(c->in_sv_off.p, sv_off, (n_docs + 1) * 8, hipMemcpyHostToDevice, c->s) != hipSuccess)
      return DEV_FAIL();
  }
  ymerge_device_result dr{};
  int st = version == 2
               ? plan_v2_device(c, diff, c->in_bytes.as<uint8_t>(), c->in_upd_off.as<uint64_t>(),
                                diff ? c->in_sv.as<uint8_t>() : nullptr, diff ? c->in_sv_off.as<uint64_t>() : nullptr,
                                n_docs, &dr)
               : plan_exec(c, diff, c->in_bytes.as<uint8_t>(), c->in_upd_off.as<uint64_t>(),
                           diff ? c->in_sv.as<uint8_t>() : nullptr, diff ? c->in_sv_off.as<uint64_t>() : nullptr,
                           n_docs, &dr, frame);
  if (st) return st;
  ymerge_batch_result *r = alloc_result(n_docs, dr.out_bytes);
  if (!r) return YMERGE_ERR_NOT_ENOUGH_MEMORY;
  st = pack_to_host(c, &dr, n_docs, r->out, r->out_off, r->status);
  if (st) {
    ymerge_batch_result_destroy(r);
    return st;
  }
  *out = r;
  return 0;
}

extern "C" int ydiff_updates_v1_batch(ymerge_ctx *c, const uint8_t *bytes, const uint64_t *upd_off,
                                      const uint8_t *sv, const uint64_t *sv_off, uint64_t n_docs,
                                      ymerge_batch_result **res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  return host_plan_exec(c, true, bytes, upd_off, sv, sv_off, n_docs, res);
}
extern "C" int ydiff_updates_v2_batch(ymerge_ctx *c, const uint8_t *bytes, const uint64_t *upd_off,
                                      const uint8_t *sv, const uint64_t *sv_off, uint64_t n_docs,
                                      ymerge_batch_result **res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  return host_plan_exec(c, true, bytes, upd_off, sv, sv_off, n_docs, res, 0, 2);
}
extern "C" int yencode_state_vector_from_update_v2_batch(ymerge_ctx *c, const uint8_t *bytes,
                                                         const uint64_t *upd_off, uint64_t n_docs,
                                                         ymerge_batch_result **res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  return host_plan_exec(c, false, bytes, upd_off, nullptr, nullptr, n_docs, res, 0, 2);
}
extern "C" int ysync_step1_v1_batch(ymerge_ctx *c, const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_docs,
                                    ymerge_batch_result **res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  return host_plan_exec(c, false, bytes, upd_off, nullptr, nullptr, n_docs, res, 2);
}
extern "C" int ysync_step2_v1_batch(ymerge_ctx *c, const uint8_t *bytes, const uint64_t *upd_off, const uint8_t *msg,
                                    const uint64_t *msg_off, uint64_t n_docs, ymerge_batch_result **res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  return host_plan_exec(c, true, bytes, upd_off, msg, msg_off, n_docs, res, 1);
}
extern "C" int yencode_state_vector_from_update_v1_batch(ymerge_ctx *c, const uint8_t *bytes,
                                                         const uint64_t *upd_off, uint64_t n_docs,
                                                         ymerge_batch_result **res) {
  if (!c || !res) return YMERGE_ERR_OTHER;
  return host_plan_exec(c, false, bytes, upd_off, nullptr, nullptr, n_docs, res);
}

static char *single_result(ymerge_batch_result *r, uint32_t *out_len) {
  if (r->status[0]) {
    g_last_error = r->status[0];
    ymerge_batch_result_destroy(r);
    return nullptr;
  }
  const uint64_t n = r->out_off[1] - r->out_off[0];
  char *res = (char *)malloc(n ? n : 1);
  if (!res) {
    g_last_error = YMERGE_ERR_NOT_ENOUGH_MEMORY;
    ymerge_batch_result_destroy(r);
    return nullptr;
  }
  memcpy(res, r->out + r->out_off[0], n);
  *out_len = (uint32_t)n;
  ymerge_batch_result_destroy(r);
  return res;
}

extern "C" char *ydiff_updates_v1(const char *update, uint32_t update_len, const char *state_vector,
                                  uint32_t sv_len, uint32_t *out_len) {
  g_last_error = 0;
  ymerge_ctx *c = default_ctx();
  if (!c) {
    g_last_error = YMERGE_ERR_DEVICE;
    return nullptr;
  }
  const uint64_t uo[2] = {0, update_len}, so[2] = {0, sv_len};
  ymerge_batch_result *r = nullptr;
  int st = ydiff_updates_v1_batch(c, (const uint8_t *)update, uo, (const uint8_t *)state_vector, so, 1, &r);
  if (st) {
    g_last_error = (uint8_t)st;
    return nullptr;
  }
  return single_result(r, out_len);
}
extern "C" char *yencode_state_vector_from_update_v1(const char *update, uint32_t update_len, uint32_t *out_len) {
  g_last_error = 0;
  ymerge_ctx *c = default_ctx();
  if (!c) {
    g_last_error = YMERGE_ERR_DEVICE;
    return nullptr;
  }
  const uint64_t uo[2] = {0, update_len};
  ymerge_batch_result *r = nullptr;
  int st = yencode_state_vector_from_update_v1_batch(c, (const uint8_t *)update, uo, 1, &r);
  if (st) {
    g_last_error = (uint8_t)st;
    return nullptr;
  }
  return single_result(r, out_len);
}

// ---------------------------------------------------------------- single document, lib0 v2
extern "C" char *ymerge_updates_v2(const char *const *updates, const uint32_t *updates_len, uint32_t updates_count,
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
  const uint64_t doc_upd[2] = {0, updates_count};
  ymerge_batch_result *r = nullptr;
  const int st = ymerge_updates_v2_batch(c, arena.data(), off.data(), updates_count, doc_upd, 1, &r);
  if (st) {
    g_last_error = (uint8_t)st;
    return nullptr;
  }
  return single_result(r, out_len);
}
extern "C" char *ydiff_updates_v2(const char *update, uint32_t update_len, const char *state_vector,
                                  uint32_t sv_len, uint32_t *out_len) {
  g_last_error = 0;
  ymerge_ctx *c = default_ctx();
  if (!c) {
    g_last_error = YMERGE_ERR_DEVICE;
    return nullptr;
  }
  const uint64_t uo[2] = {0, update_len}, so[2] = {0, sv_len};
  ymerge_batch_result *r = nullptr;
  const int st = ydiff_updates_v2_batch(c, (const uint8_t *)update, uo, (const uint8_t *)state_vector, so, 1, &r);
  if (st) {
    g_last_error = (uint8_t)st;
    return nullptr;
  }
  return single_result(r, out_len);
}
extern "C" char *yencode_state_vector_from_update_v2(const char *update, uint32_t update_len, uint32_t *out_len) {
  g_last_error = 0;
  ymerge_ctx *c = default_ctx();
  if (!c) {
    g_last_error = YMERGE_ERR_DEVICE;
    return nullptr;
  }
  const uint64_t uo[2] = {0, update_len};
  ymerge_batch_result *r = nullptr;
  const int st = yencode_state_vector_from_update_v2_batch(c, (const uint8_t *)update, uo, 1, &r);
  if (st) {
    g_last_error = (uint8_t)st;
    return nullptr;
  }
  return single_result(r, out_len);
}

extern "C" void ymerge_binary_destroy(char *ptr, uint32_t) { free(ptr); }
// yffi-compatible name for processes that link this library alone.  Next to yffi the
// dynamic linker binds it to the first DSO in lookup order (weak does not lose to strong
// across shared objects), so include/ymerge.h names ymerge_binary_destroy as the only safe
// free for this library's buffers.
extern "C" __attribute__((weak)) void ybinary_destroy(char *ptr, uint32_t len) { ymerge_binary_destroy(ptr, len); }
