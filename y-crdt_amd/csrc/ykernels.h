// ykernels.h — launch interface between the host engine (ymerge_host.cpp) and the
// gfx950 kernels.  Plain device pointers only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ym {
// exclusive scan: out[0..n] (out[n] = total); tmp needs >= (n/2048 + 2) u64
// n_dev: optional device-side element count (<= n, the count the grid is sized for)
void launch_scan_u64(const uint64_t *in, uint64_t *out, uint32_t n, uint64_t *tmp, hipStream_t s,
                     const uint32_t *n_dev = nullptr);
// A batch of documents in HBM: doc d owns updates [doc_upd[d], doc_upd[d+1]);
// update u owns bytes [upd_off[u], upd_off[u+1]) of `bytes`.
struct BatchIn {
  const uint8_t *bytes;
  const uint64_t *upd_off;
  const uint64_t *doc_upd;
  uint32_t n_docs;
  const uint32_t *rec; // per-update decode records (k_decode), REC_WORDS u32 each; fast path only
  const uint32_t *ovf; // their overflow words (DEC_OVF per decode workgroup)
  uint32_t v1x = 0;    // bytes are the internal v1x grammar (lib0 v2 path), not lib0 v1
  uint32_t only_path3 = 0; // k_fast_merge: only the documents k_lean handed over (path == 3)
  const uint32_t *order = nullptr; // k_lean: wavefront -> document (long documents first), or identity
  uint32_t lean_umax = 0;          // k_lean: hand over documents of more updates (0: LN_UMAX)
};

// Per-update decode record written by k_decode (one lane per update over the whole
// batch) and consumed by k_fast_merge.  w0 = error code (bits 0-7) | REC_UNSUP |
// REC_BIGDS | shape << 10 | DeleteSet ranges << 12 | REC_SLOW (needs the exact walk,
// done by k_fast_merge); then by shape
//   REC_BLOCK   : client, clock, length, byte position within the update, meta
//   REC_DS      : client, start0, end0, start1, end1 (one DeleteSet entry, <= 2 ranges)
//   REC_COMPLEX : blocks, entries, ranges, [REC_OVF: word offset of its records in the
//                 overflow buffer (OvfFill layout), else the fast kernel walks it again]
constexpr uint32_t DEC_NT = 256, DEC_STAGE = 16384, DEC_OVF = 1024; // overflow words per decode workgroup
constexpr uint32_t REC_WORDS = 6;
constexpr uint32_t REC_UNSUP = 1u << 8, REC_BIGDS = 1u << 9, REC_SLOW = 1u << 14, REC_OVF = 1u << 15;
constexpr uint32_t REC_EMPTY = 0, REC_BLOCK = 1, REC_DS = 2, REC_COMPLEX = 3;
// huge: [count, exact-walker count, u64 overflow bump, u64 list of HUGE_LIST update indices];
// huge_cap: overflow words after the k_decode workgroups' DEC_OVF words for the long updates
constexpr uint32_t HUGE_LIST = 65536;
// an update k_decode could not stage: >= LP_MIN_LEN bytes -> the parallel parse (ylong.hip),
// shorter ones -> k_decode_exact's later staging rounds
constexpr uint32_t LP_MIN_LEN = 8192;
// a staged update of >= LP_MID_LEN bytes the fast walk cannot take goes to the parallel parse too:
// the exact walk is one wavefront stepping serially (~1,800 cycles a varint), a 5 KB rich update
// ~6 ms of one workgroup's time (env YMERGE_LP_MID)
constexpr uint32_t LP_MID_LEN = 128;
constexpr uint32_t LP_EXT_T = 1024; // positions per k_lp_ext tile
// and every update of >= LP_DIRECT_LEN bytes, without the fast lane walk first
constexpr uint32_t LP_DIRECT_LEN = 1024;
// k_decode workgroups with staged updates for the exact walk (k_decode_exact): count at word
// EXQ_COUNT of `huge`, then (workgroup, overflow words used) pairs, one per decode workgroup
constexpr uint32_t EXQ_COUNT = 4 + 2 * HUGE_LIST, EXQ_LIST = EXQ_COUNT + 4;
inline uint64_t huge_bytes(uint64_t n_updates) { return 4ull * EXQ_LIST + 8 * ((n_updates + DEC_NT - 1) / DEC_NT + 1); }
constexpr uint32_t REC_STAGED = 1u << 17; // with REC_SLOW: walked exactly by k_decode_exact (LDS stage)
// REC_COMPLEX record written by the parallel long-update parse (ylong.hip) for an update of one
// client section without Skips, zero-length GC blocks, panicking splits or unsupported content,
// and <= 1 DeleteSet entry; w5 = its LP entry + 1 (grid paths for single-update documents)
constexpr uint32_t REC_LONG = 1u << 16;
// a client section whose client is not below the previous section's: decoding appends a repeated
// client's sections to one block queue in section order (yrs/src/update.rs:714-749), which the
// sort-based paths (fast, tiled, grid) do not model; such documents go to the exact engine
// (encoders write sections in descending client order, so valid updates never carry it)
constexpr uint32_t REC_ORDER = 1u << 18;

// ---- parallel parse of long updates (ylong.hip)
constexpr uint32_t LP_CH = 8192;  // bytes per chunk
constexpr uint32_t LP_MW = 16;    // meta words per long update
constexpr uint32_t LP_SEGW = 6;   // words per segment
enum : uint32_t {                 // meta words
  LPM_U = 0, LPM_L = 2, LPM_CB, LPM_NCH, LPM_PB, LPM_FLAGS, LPM_NBALL, LPM_NB, LPM_DS, LPM_SB, LPM_NCL, LPM_OB, LPM_OVF,
  LPM_NE, LPM_NR
};
enum : uint32_t { // flags
  LPF_FALLBACK = 1, LPF_UNSUP = 2, LPF_SKIP = 4, LPF_ZGC = 8, LPF_PANIC = 16, LPF_MSEC = 32, LPF_RICH = 64, LPF_ORDER = 128
};
enum : uint32_t { LPG_CHUNKS = 0, LPG_SEGS, LPG_ORDS, LPG_SECS, LPG_N, LPG_TILES, LPG_WORDS = 8 };
struct LpArgs {
  const uint8_t *bytes;
  const uint64_t *upd_off;
  uint32_t *rec, *ovf;
  uint32_t *huge;            // k_decode's list: [0] count, [1] exact-walker count, [2..3] u64 overflow bump, list
  uint32_t huge_base;        // first overflow word of the long-update region
  uint64_t huge_cap;         // its words
  uint32_t *meta, *g, *c2e;  // per long update, counters, chunk -> update
  uint32_t *ext;             // [pcap] speculative block ends
  uint64_t *jc;              // [pcap] (first boundary past the chunk, blocks | stored << 16)
  uint32_t *seg, *sec;       // segments [scap], sections [seccap] (client, clock, first ordinal, update)
  uint64_t *blen, *sblen;    // [ocap] clock lengths in block order, scan [ocap + 1]
  uint32_t *omap;            // [ocap] record word + 1 of a stored block, 0 otherwise
  uint64_t *fb;              // updates left to the exact walker (k_decode_huge)
  uint64_t *tmap;            // [tcap] k_lp_ext tiles: (entry << 32) | tile within the entry
  uint64_t *scan_tmp;
  uint32_t pcap, ccap, scap, seccap, ocap, tcap;
  uint32_t v1x;
  uint32_t mid; // k_decode lists updates of >= mid bytes its fast walk cannot take (LP_MID_LEN)
};
void launch_long_decode(const LpArgs &a, hipStream_t s);

// ---- single long update documents on the grid (ylong.hip, after the parallel parse): merge_updates_v1
// of a document that is one REC_LONG update, its diff_updates_v1 / state vector.  One document
// per launch sequence; the list entries (LS_EW words) come from k_ls_find / k_ls_collect.
constexpr uint32_t LS_LIST = 16, LS_EW = 8; // entry: doc, update lo, hi, L, NB, NE, NR, ovf base
constexpr uint32_t LS_MIN_DIFF = 65536;     // diff / SV: documents of >= this many bytes (env YMERGE_LS_MIN)
enum : uint32_t { LSG_BAD = 0, LSG_K0, LSG_OFF, LSG_HDR, LSG_DSH, LSG_K, LSG_CLIENT, LSG_CLOCK, LSG_END, LSG_WORDS = 16 };
struct LsArgs {
  const uint8_t *bytes;    // the update: bytes + upd_off[u]
  uint32_t L, NB, NE, NR;
  const uint32_t *ov;      // its records (OvfFill layout)
  uint32_t d, mode;        // document; 0 merge, 1 diff, 2 state vector
  uint32_t v1x, frame;     // grammar; y-sync framing (diff / SV)
  const uint8_t *sv;       // diff: remote state vector bytes
  const uint64_t *sv_off, *sv_end;
  uint32_t *g;             // LSG_WORDS per document
  uint64_t *bsz, *boff;    // [NB], [NB + 1]
  uint64_t *rsz, *roff;    // [NR], [NR + 1] (merge: run starts, run indices)
  uint64_t *rsz2, *roff2;  // merge: [NR], [NR + 1] run sizes, offsets
  uint32_t *rstart, *rend; // merge: [NR] run starts / ends
  uint64_t *scan_tmp;
  // merge: the document's slot in the output arena; diff / SV: the packed output (after the scan)
  uint8_t *out;
  const uint64_t *upd_off; // (merge: the slot is 2 * upd_off[u] + 64 * d)
  uint64_t u;
  uint64_t *out_start, *out_len, *size;
  uint8_t *status, *path, *done;
  uint32_t *npath;
  const uint64_t *pack_off;
};
void launch_ls_find(const BatchIn &b, const uint8_t *path, uint32_t *list, hipStream_t s);
void launch_ls_list_diff(const uint64_t *upd_off, const uint8_t *pre_status, uint32_t n_docs, uint32_t min_len,
                         uint32_t *huge, hipStream_t s);
void launch_ls_collect(const LpArgs &a, uint32_t *list, hipStream_t s);
// phase 0: checks, sizes, scans, totals (merge: also the write); phase 1 (diff / SV): the write
void launch_ls_doc(const LsArgs &a, int phase, hipStream_t s);
void launch_decode(const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_updates, uint32_t *rec, uint32_t *ovf,
                   uint32_t *huge, uint32_t huge_cap, hipStream_t s, const LpArgs *lp = nullptr, uint32_t v1x = 0,
                   uint64_t *dbg = nullptr,
                   uint32_t *h_probe = nullptr);

// LDS capacities of the one-workgroup-per-document fast path (per document)
struct FastCaps {
  uint32_t in_cap, u_cap, b_cap, e_cap, r_cap;
  uint32_t ident = 1; // single-update identity copy (env YMERGE_IDENTITY=0: off)
};
// per-document results; path 0 = written, 1 = needs the exact engine, 2 = needs the tiled
// kernel for documents above the LDS capacities
struct FastOut {
  uint8_t *out; // output arena: document d's slot starts at 2*byte_start(d) + 64*d
  uint64_t *out_start, *out_len;
  uint8_t *status, *path;
  uint64_t *stamps; // diagnostic build only: s_memtime per phase (16 per document)
  uint32_t *dbg = nullptr; // k_lean diagnostics (env YMERGE_LEAN_DEBUG): 8 words per document
  uint32_t *npath;  // npath[p]: documents handed to path p (1 exact engine, 2 tiled kernel); [3] tiled
                    // kernel in overlap mode, [4] tiled kernel -> exact engine, [5] of [1]:
                    // tiny documents (FastCaps.in_cap / u_cap), [6] k_lean -> fast path,
                    // [7..13] k_lean hand-over reasons
  unsigned long long *lean_total = nullptr; // k_lean output bytes: 64 partial sums, 8 words apart
  uint32_t *big_list = nullptr; // [n_docs]: the documents handed to path 2, in npath[2] order
};
size_t fast_lds_bytes(const FastCaps &c);
// one wavefront per document for the common editor shape (ymerge_lean.hip): writes the
// document (path 0) or hands it to k_decode + k_fast_merge (path 3, counted in npath[6]).
// scr: HBM scratch of lean_scratch_words(...) u32 for documents above the LDS arena (null:
// those are handed over)
void launch_lean(const BatchIn &b, const FastOut &o, uint32_t *scr, hipStream_t s);
// after k_lean: its hand-over count (counter word 10) and the sum of its 64 output-byte
// partials (from word 32, 16 words apart) to the host-mapped sig[1..3], then sig[0] = seq;
// with no hand-over it zeroes counter words [0, 32 + 1024) for the next merge
void launch_lean_fin(uint32_t *counter, uint32_t *sig, uint32_t seq, hipStream_t s);
// k_lean dispatch order for skewed batches: documents by update-count class, longest class
// first (longest-processing-time-first: a long document starts early instead of ending the
// kernel).  ctr: 16 zeroed words.
void launch_lean_order(const uint64_t *doc_upd, uint32_t n_docs, uint32_t *ctr, uint32_t *order, hipStream_t s);
inline uint64_t lean_scratch_words(uint64_t n_updates, uint64_t n_docs, uint64_t n_bytes) {
  return 4 * n_updates + 64 * n_docs + n_bytes;
}
void launch_fast_merge(const BatchIn &b, const FastCaps &caps, const FastOut &o, int nt, hipStream_t s);
// one long single-client document merged by grid-wide kernels (ygiant.hip)
constexpr uint32_t GS_LIST = 16;     // such documents per batch (the rest: tiled kernel)
constexpr uint32_t GS_MIN_U = 8192; // updates (env YMERGE_GIANT_MIN; editing traces: 4 of 5 documents on the grid path)
// batches of <= GS_SMALL_DOCS documents (too few for k_lean's waves to fill the GPU): documents
// of >= GS_MIN_SMALL updates skip k_lean (one wave serially: friendsforever_flat's 4,288
// updates took 0.40 ms) and take the grid path when they are its shape
constexpr uint32_t GS_SMALL_DOCS = 64, GS_MIN_SMALL = 4096;
constexpr uint8_t GS_PATH = 5;       // path of a listed document until k_gs_final decides
struct GsArgs {
  const uint8_t *bytes;
  const uint64_t *upd_off;
  const uint32_t *rec, *ovf;
  uint64_t u0;
  uint32_t U, d;
  uint8_t *out; // the output arena (the document's slot is 2 x its first byte + 64 x d, on the device)
  uint64_t *cnt, *bl;    // [U]: blocks | ranges << 32, block bytes << 32 | clock lengths
  uint64_t *s_cnt, *s_bl; // [U + 1] exclusive scans
  uint32_t *g;                         // flags / client min, max / max range end / first block key
  uint32_t *gp;                        // k_gs_pre's per-workgroup partials of g (6 words each)
  uint32_t *bm;                        // deleted-clock bitmap [nwords]
  uint32_t nbits, nwords;              // bitmap capacity (bits, words); the words in use are on the device
  uint32_t kcap;                       // squashed-range capacity
  uint64_t *w_cnt, *w_scan;            // run starts per word, scan [nwords + 1]
  uint32_t *k_start, *k_len;           // runs = squashed ranges
  uint64_t *k_size, *k_off;
};
void launch_gs_find(const BatchIn &b, uint8_t *path, uint32_t min_u, uint64_t *list, hipStream_t s);
void launch_gs_pre(const GsArgs &a, hipStream_t s);
void launch_gs_rest(const GsArgs &a, const FastOut &o, uint64_t *scan_tmp, hipStream_t s);

// store-based compaction (ycompact.hip): one lane per document applies its updates to a
// device block store; documents outside the device shape get status E_UNSUPPORTED.
// k_compact_count fills a 32-word header per document and its scratch words (need[d]);
// scr_off = exclusive scan of need (n_docs + 1 entries)
constexpr uint32_t COMPACT_HDR_WORDS = 40; // ycompact.hip CP_HDR (16 clients)
void launch_compact_count(const BatchIn &b, uint32_t *hdr, uint64_t *need, hipStream_t s);
void launch_compact(const BatchIn &b, const FastOut &o, uint32_t *hdr, const uint64_t *scr_off, uint32_t *scr,
                    uint32_t lpw, hipStream_t s);

// documents over the fast path's LDS capacities (path == 2): tiled, HBM scratch
// over o.big_list[0, n_list) (need[] of the other documents must be zero)
void launch_big_count(const BatchIn &b, const FastOut &o, uint32_t *counts, uint64_t *need, uint32_t *n_big,
                      uint32_t n_list, hipStream_t s);
void launch_big_merge(const BatchIn &b, const uint32_t *counts, const uint64_t *scr_off, uint32_t *scratch,
                      const FastOut &o, uint32_t n_list, hipStream_t s);

// exact per-document engine; `path` (optional) restricts it to documents with path == 1; lpw
// documents per wavefront (1..64)
void launch_seq_count(const BatchIn &b, const uint8_t *path, uint8_t *status, uint32_t *counts, uint64_t *need,
                      uint32_t *n_exact, hipStream_t s, uint32_t lpw = 64);
void launch_seq_merge(bool write, const BatchIn &b, const uint8_t *path, const uint8_t *status, const uint32_t *counts,
                      const uint64_t *scr_off, uint32_t *scratch, uint64_t *sizes, const uint64_t *out_off,
                      uint8_t *out, uint64_t out_base, uint64_t *out_start, uint64_t *out_len, uint8_t *status_out,
                      hipStream_t s, uint32_t lpw = 64, uint64_t *dbg = nullptr);
size_t scan_tmp_elems(uint32_t n);
void launch_pack(const uint8_t *src, const uint64_t *start, const uint64_t *len, const uint64_t *pack_off,
                 uint8_t *dst, uint32_t n_docs, hipStream_t s);
// a[i] -= sub for i < n (offset tables of a pipelined host group, rebased to the group's slice)
void launch_rebase_u64(uint64_t *a, uint64_t n, uint64_t sub, hipStream_t s);
} // namespace ym

namespace ym {
// ---- diff_updates_v1 / encode_state_vector_from_update_v1 (ydiff.hip): one update per document
struct DiffBatch {
  const uint8_t *bytes;
  const uint64_t *upd_off; // n_docs + 1
  const uint8_t *sv;       // remote state vectors (diff only)
  const uint64_t *sv_off;  // n_docs + 1 (diff only)
  uint32_t n_docs;
  const uint64_t *sv_end = nullptr;       // optional: doc d's SV is [sv_off[d], sv_end[d])
  const uint8_t *pre_status = nullptr;    // optional: nonzero = the document failed before planning
  uint32_t frame = 0;                     // y-sync framing: 0 none, 1 SyncStep2, 2 SyncStep1
  uint32_t v1x = 0;                       // bytes are the internal v1x grammar (lib0 v2 path)
  const uint8_t *ls_done = nullptr;       // optional: nonzero = planned and written by the long-update grid path
};
// y-sync: parse one client message per document (must be Message::Sync(SyncStep1(sv)),
// yrs/src/sync/protocol.rs:179-203, 245-272) -> SV slice [sv_off, sv_end) + status
// lib0 v2 (yv2.hip): v2 -> v1x transcode per update, per-document status fixup, state
// vector header parse, v1x -> v2 encode per document (mode 0 update, 1 state vector)
void launch_v2_decode(bool write, const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_upd, uint64_t *sz_off,
                      uint8_t *out, uint8_t *ust, hipStream_t s);
void launch_v2_doc_status(const uint64_t *doc_upd, const uint8_t *ust, uint32_t n_docs, uint8_t *status,
                          uint64_t *out_len, hipStream_t s);
void launch_v2_sv_parse(const uint8_t *sv, const uint64_t *sv_off, const uint8_t *ust, uint32_t n, uint64_t *rest_off,
                        uint64_t *rest_end, uint8_t *pre, hipStream_t s);
void launch_v2_encode(bool write, const uint8_t *src, const uint64_t *src_start, const uint64_t *src_len,
                      const uint8_t *status, uint32_t n_docs, uint64_t *sz_off, uint8_t *out, int mode, hipStream_t s);
// one-pass EncoderV2 (full updates): per-document column streams in scr (11 x (2 len + 64)
// bytes at scr_off, scanned from need), column sizes (11 u32 per document), document sizes;
// *over != 0: a column outgrew its stream (run the writing walk instead of k_v2_pack)
void launch_v2_encode_one(const uint8_t *src, const uint64_t *src_start, const uint64_t *src_len, const uint8_t *status,
                          uint32_t n_docs, uint64_t *need, uint64_t *scr_off, uint64_t *scan_tmp, uint8_t *scr,
                          uint32_t *colsz, uint64_t *sz, uint32_t *over, hipStream_t s);
// one-pass DecoderV2: v1x bytes of update u into scr at 4 (upd_off[u] - upd_off[0]) + 64 u
// (4 len + 64 bytes), sizes; *over != 0: a slot overflowed (run the two walks instead)
void launch_v2_decode_one(const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_upd, uint8_t *scr, uint64_t *sz,
                          uint8_t *ust, uint32_t *over, hipStream_t s);
void launch_v2_xpack(const uint64_t *upd_off, uint64_t n_upd, const uint8_t *scr, const uint64_t *off, uint8_t *out,
                     hipStream_t s);
void launch_v2_pack(const uint64_t *src_len, const uint8_t *status, uint32_t n_docs, const uint64_t *scr_off,
                    const uint8_t *scr, const uint32_t *colsz, const uint64_t *out_off, uint8_t *out, hipStream_t s);
void launch_sync_parse(const uint8_t *msg, const uint64_t *msg_off, uint32_t n, uint64_t *sv_off, uint64_t *sv_end,
                       uint8_t *status, hipStream_t s);
struct PlanCaps {
  uint32_t C, E, R, O; // client sections, DeleteSet entries, squash ranges, output ops
};
struct PlanScratch {
  uint32_t *small;        // n_docs * small_words
  uint64_t small_words;
  uint32_t *bigscr;       // documents re-planned with capacities sized from their length
  const uint64_t *big_off; // word offset per document into bigscr
  uint8_t *big, *status;
  uint64_t *size;
  uint32_t *n_big;
  uint64_t *stamps = nullptr; // diagnostic (env YMERGE_STAMPS): k_plan_ring phase cycles, 16 per document
  uint32_t planner = 0;        // pass 0 common-shape planner: 0 k_plan_lane (+ k_plan_wave for long updates),
                               // 1 k_plan_ring, 2 k_plan_wave for every document (env YMERGE_PLANNER=ring|wave)
  uint32_t *wave_list = nullptr; // planner 0: documents k_plan_lane leaves to k_plan_wave (n_docs words)
  uint32_t *wave_n = nullptr;    // ... and their count (zeroed before the launch)
  uint32_t lane_dbg = 0;         // k_plan_lane diagnostics (env YMERGE_LANE_DBG): 1 no fast step, 2 no wave DeleteSet
};
uint64_t plan_small_words();
void launch_plan(bool diff, int pass, const DiffBatch &b, const PlanScratch &ps, hipStream_t s);
void launch_big_need(const uint64_t *upd_off, const uint8_t *big, uint32_t n, uint64_t *need, hipStream_t s);
void launch_exec(const DiffBatch &b, const PlanScratch &ps, const uint64_t *out_off, uint8_t *out, hipStream_t s);
} // namespace ym
