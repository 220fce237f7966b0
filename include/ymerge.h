/*
 * ymerge.h — C ABI of the MI355X batched Yjs update-compaction engine.
 *
 * Drop-in boundary for yrs' binary-update algebra (lib0 v1):
 *   ymerge_updates_v1                  replaces yrs::merge_updates_v1                 yrs/src/alt.rs:15-28
 *   ydiff_updates_v1                   replaces yrs::diff_updates_v1                  yrs/src/alt.rs:73-81
 *   yencode_state_vector_from_update_v1 replaces yrs::encode_state_vector_from_update_v1 yrs/src/alt.rs:54-57
 *   ymerge_binary_destroy              same contract as yffi's ybinary_destroy       yffi/src/lib.rs:384-388
 *   ybinary_destroy                    weak alias of ymerge_binary_destroy (see below)
 * yffi in this snapshot exports no merge/diff-of-updates function;
 * the signatures follow yffi conventions: `const char *` + `uint32_t` length
 * inputs, a library-owned `char *` result with its length in `*out_len`, NULL on
 * a decode failure (yffi/src/lib.rs:802-829), error codes as yffi's
 * (yffi/src/lib.rs:1137-1174): 2 VAR_INT, 3 EOS, 4 UNEXPECTED_VALUE, 5 INVALID_JSON,
 * 6 OTHER, 7 NOT_ENOUGH_MEMORY, plus 20 REFERENCE_PANIC (yrs panics, or overflows u32
 * clock arithmetic that only a debug build checks: see INTEGRATION.md)
 * and 21 UNSUPPORTED (content class not restated on the device yet).
 *
 * Batched entry points take one contiguous byte arena for many documents:
 * doc d owns updates [doc_upd[d], doc_upd[d+1]), update u owns bytes
 * [upd_off[u], upd_off[u+1]).  Each document's output equals the single-document
 * function on that document's updates.
 *
 * Thread safety: every function is safe to call concurrently; a ymerge_ctx
 * serialises the batches submitted to it on its own HIP stream.
 */
#ifndef YMERGE_H
#define YMERGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YMERGE_OK 0
#define YMERGE_ERR_VAR_INT 2
#define YMERGE_ERR_EOS 3
#define YMERGE_ERR_UNEXPECTED_VALUE 4
#define YMERGE_ERR_INVALID_JSON 5
#define YMERGE_ERR_OTHER 6
#define YMERGE_ERR_NOT_ENOUGH_MEMORY 7
#define YMERGE_ERR_REFERENCE_PANIC 20
#define YMERGE_ERR_UNSUPPORTED 21
#define YMERGE_ERR_DEVICE 30 /* no usable MI355X / HIP failure */

/* ---------------------------------------------------------------- single document (yffi style) */
char *ymerge_updates_v1(const char *const *updates, const uint32_t *updates_len, uint32_t updates_count,
                        uint32_t *out_len);
char *ydiff_updates_v1(const char *update, uint32_t update_len, const char *state_vector, uint32_t sv_len,
                       uint32_t *out_len);
char *yencode_state_vector_from_update_v1(const char *update, uint32_t update_len, uint32_t *out_len);
/* lib0 v2 forms: yrs::merge_updates_v2 / diff_updates_v2 / encode_state_vector_from_update_v2
 * (yrs/src/alt.rs:35-48, 88-97, 63-66) */
char *ymerge_updates_v2(const char *const *updates, const uint32_t *updates_len, uint32_t updates_count,
                        uint32_t *out_len);
char *ydiff_updates_v2(const char *update, uint32_t update_len, const char *state_vector, uint32_t sv_len,
                       uint32_t *out_len);
char *yencode_state_vector_from_update_v2(const char *update, uint32_t update_len, uint32_t *out_len);
/* frees a buffer returned by the three calls above */
void ymerge_binary_destroy(char *ptr, uint32_t len);
/* yffi's name, exported as a WEAK symbol for processes that link this library alone.
 * When yffi is loaded too, the dynamic linker binds the name to whichever shared object
 * comes first in lookup order (glibc does not rank weak below strong across DSOs), so
 * which library's buffers it frees depends on link/load order: ymerge_binary_destroy is
 * the only safe way to free this library's buffers. */
void ybinary_destroy(char *ptr, uint32_t len);
/* error code of the last failed call on this thread (0 after a success) */
uint8_t ymerge_last_error(void);
/* where the last YMERGE_ERR_DEVICE on this thread came from: the failing stage and the HIP
 * error string (empty before any device failure; valid until the next one on the thread) */
const char *ymerge_last_error_message(void);
/* device of the single-document calls (default: env YMERGE_DEVICE, else 0);
 * returns 0 or YMERGE_ERR_DEVICE for a device that does not exist */
int ymerge_set_default_device(int device);

/* ---------------------------------------------------------------- batched, device-resident */
typedef struct ymerge_ctx ymerge_ctx;
ymerge_ctx *ymerge_ctx_create(int device);
void ymerge_ctx_destroy(ymerge_ctx *ctx);

/* Per-batch statistics (device event timings of the last batch, ms). */
typedef struct {
  uint64_t n_docs, bytes_in, bytes_out;
  uint64_t docs_fast, docs_exact, docs_error;
  float ms_total, ms_fast, ms_exact, ms_tail;
  float ms_decode; /* merge: k_decode (ms_fast = k_fast_merge only) */
  float ms_big;    /* merge: documents over the LDS capacities (k_big_count + k_big_merge) */
  uint32_t docs_overlap; /* merge: of docs_big, documents with overlapping updates (run order, splices) */
  uint64_t docs_big; /* merge: documents written by the tiled kernel or the grid-wide kernels
                        (docs_giant; docs_exact: exact engine) */
  uint64_t docs_tiny; /* merge: documents of <= 4 updates (<= 4 KB) written one lane each by the
                         lane-per-document engine (not counted in docs_exact) */
  float ms_tiny;      /* merge: exact-engine stage time when it ran tiny documents only */
  uint64_t docs_lean; /* merge: documents written by k_lean (one wavefront each; not in docs_fast) */
  float ms_lean;      /* merge: k_lean (ms_decode / ms_fast then time the documents it handed over) */
  uint64_t docs_giant; /* merge: of docs_big, long single-client documents merged by the grid-wide
                          kernels of ygiant.hip instead of one tiled workgroup */
  float ms_v2_decode, ms_v2_merge, ms_v2_encode; /* merge_updates_v2: the v2 -> v1x transcode, the v1
                          pipeline, the v2 encode (incl. their host syncs) */
} ymerge_stats;

/* Device-resident result, owned by the context, valid until the next batch.
 * Document d's output is d_out[d_out_start[d] .. d_out_start[d] + d_out_len[d]);
 * documents are written where their slot is (no packing pass on the hot path). */
typedef struct {
  uint8_t *d_out;         /* output arena */
  uint64_t *d_out_start;  /* n_docs */
  uint64_t *d_out_len;    /* n_docs (0 when status != 0) */
  uint8_t *d_status;      /* n_docs status codes */
  uint64_t arena_bytes;   /* size of d_out */
  uint64_t out_bytes;     /* sum of d_out_len */
} ymerge_device_result;

/* merge_updates_v1 over a batch whose arena (n_bytes) and offsets (n_updates + 1,
 * n_docs + 1) already live in HBM of the context's device.  The kernels load the arena
 * in aligned 4/16-byte words: d_bytes must be 16-byte aligned (hipMalloc's are) and stay
 * readable for 16 bytes past n_bytes (pad the allocation; the host entry points do).  Same
 * for the update/SV arenas below.
 * Returns 0 or YMERGE_ERR_DEVICE. */
int ymerge_updates_v1_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes, uint64_t n_bytes,
                                   const uint64_t *d_upd_off, uint64_t n_updates, const uint64_t *d_doc_upd,
                                   uint64_t n_docs, ymerge_device_result *res);
/* encode_state_vector_from_update_v1 / diff_updates_v1: one update per document
 * (d_upd_off has n_docs + 1 entries); diff also takes one encoded state vector
 * per document. */
int yencode_state_vector_from_update_v1_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes,
                                                     const uint64_t *d_upd_off, uint64_t n_docs,
                                                     ymerge_device_result *res);
int ydiff_updates_v1_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                                  const uint8_t *d_sv_bytes, const uint64_t *d_sv_off, uint64_t n_docs,
                                  ymerge_device_result *res);
/* y-sync serving over the update algebra (yrs/src/sync/protocol.rs:62-69, 219-272), one
 * compacted update per document:
 *  ysync_step1_v1_*: Message::Sync(SyncStep1(sv)).encode = [0, 0, varbuf(sv)] with
 *    sv = encode_state_vector_from_update_v1(update);
 *  ysync_step2_v1_*: decodes each document's client message, which must be
 *    Message::Sync(SyncStep1(remote sv)) (document d's message is msg[msg_off[d] ..
 *    msg_off[d+1]); other messages -> status UNSUPPORTED, malformed ones the decode error),
 *    and answers Message::Sync(SyncStep2(diff_updates_v1(update, remote sv))) =
 *    [0, 1, varbuf(diff)]: what Protocol::handle_sync_step1 replies. */
int ysync_step1_v1_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes, const uint64_t *d_upd_off, uint64_t n_docs,
                                ymerge_device_result *res);
int ysync_step2_v1_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                                const uint8_t *d_msg, const uint64_t *d_msg_off, uint64_t n_docs,
                                ymerge_device_result *res);
/* lib0 v2 (yrs/src/alt.rs:35-48, 63-66, 88-97): the same operations over v2-encoded updates
 * and state vectors (yrs/src/updates/{decoder,encoder}.rs), outputs v2-encoded.  Device
 * limits (status UNSUPPORTED): client ids >= 2^32; a key-table hit beyond the first 64 keys
 * of one update. */
int ymerge_updates_v2_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes, uint64_t n_bytes,
                                   const uint64_t *d_upd_off, uint64_t n_updates, const uint64_t *d_doc_upd,
                                   uint64_t n_docs, ymerge_device_result *res);
int ydiff_updates_v2_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes, const uint64_t *d_upd_off,
                                  const uint8_t *d_sv_bytes, const uint64_t *d_sv_off, uint64_t n_docs,
                                  ymerge_device_result *res);
int yencode_state_vector_from_update_v2_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes,
                                                     const uint64_t *d_upd_off, uint64_t n_docs,
                                                     ymerge_device_result *res);
/* Store-based compaction: document d's updates applied in order to a fresh
 * yrs Doc with GC on, one transaction each (yffi ytransaction_apply, yffi/src/lib.rs:1078;
 * TransactionMut::apply_update, yrs/src/transaction.rs:675-730), then the whole state encoded
 * (ytransaction_state_diff_v1 with no state vector, yffi/src/lib.rs:802; Doc
 * encode_state_as_update_v1, yrs/src/transaction.rs:73-85): squashed Items, GC'd content.
 * Device shape (ycompact.hip header); documents outside it get status YMERGE_ERR_UNSUPPORTED
 * (21), decode errors their yrs code. */
int ycompact_updates_v1_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes, uint64_t n_bytes,
                                     const uint64_t *d_upd_off, uint64_t n_updates, const uint64_t *d_doc_upd,
                                     uint64_t n_docs, ymerge_device_result *res);
/* lib0 v1 -> v2 of every update of an arena: each update u becomes
 * merge_updates_v1([u]) re-encoded by EncoderV2 (yrs/src/alt.rs:15-28 then
 * Update::encode_v2, yrs/src/updates/encoder.rs:182-528).  For a canonical update this equals
 * Update::decode_v1(u).encode_v2(); they differ where merge itself rewrites a single update
 * (overlapping same-client blocks sliced, adjacent Skips joined, update.rs:611-679, 854) and
 * merge-only rejections give a nonzero status.  res lists one v2 update per input update.
 * Feeds the v2 entry points (bench, tests). */
int yconvert_updates_v1_to_v2_batch_device(ymerge_ctx *ctx, const uint8_t *d_bytes, uint64_t n_bytes,
                                           const uint64_t *d_upd_off, uint64_t n_updates,
                                           ymerge_device_result *res);
/* pack the last device result into host buffers: out (res->out_bytes), out_off (n_docs + 1,
 * document d at out[out_off[d] .. out_off[d+1])), status (n_docs) */
int ymerge_result_to_host(ymerge_ctx *ctx, const ymerge_device_result *res, uint64_t n_docs, uint8_t *out,
                          uint64_t *out_off, uint8_t *status);
void ymerge_last_stats(ymerge_ctx *ctx, ymerge_stats *stats);
/* stage timing (the ms_* fields of ymerge_last_stats: HIP events around the stages), on by
 * default.  Off (on = 0): a merge that k_lean writes whole records no events (one host call
 * less per event on its critical path; its ms_* read 0).  Results are the same either way. */
void ymerge_ctx_set_stage_timing(ymerge_ctx *ctx, int on);
/* diagnostic builds (env YMERGE_STAMPS=1): per-document s_memtime phase stamps, 16 per doc */
int ymerge_debug_stamps(ymerge_ctx *ctx, uint64_t n_docs, uint64_t *dst);

/* ---------------------------------------------------------------- batched, host memory */
typedef struct {
  uint8_t *out;      /* library-owned arena */
  uint64_t *out_off; /* n_docs + 1 */
  uint8_t *status;   /* n_docs */
  uint64_t n_docs, out_bytes;
} ymerge_batch_result;
int ymerge_updates_v1_batch(ymerge_ctx *ctx, const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_updates,
                            const uint64_t *doc_upd, uint64_t n_docs, ymerge_batch_result **res);
/* diff_updates_v1 over a batch: document d = one update bytes[upd_off[d] .. upd_off[d+1]) and one
 * encoded remote state vector sv[sv_off[d] .. sv_off[d+1]) (sync-step-2 serving, yrs/src/alt.rs:73-81) */
int ydiff_updates_v1_batch(ymerge_ctx *ctx, const uint8_t *bytes, const uint64_t *upd_off, const uint8_t *sv,
                           const uint64_t *sv_off, uint64_t n_docs, ymerge_batch_result **res);
/* encode_state_vector_from_update_v1 over a batch (yrs/src/alt.rs:54-57) */
int yencode_state_vector_from_update_v1_batch(ymerge_ctx *ctx, const uint8_t *bytes, const uint64_t *upd_off,
                                              uint64_t n_docs, ymerge_batch_result **res);
int ysync_step1_v1_batch(ymerge_ctx *ctx, const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_docs,
                         ymerge_batch_result **res);
int ysync_step2_v1_batch(ymerge_ctx *ctx, const uint8_t *bytes, const uint64_t *upd_off, const uint8_t *msg,
                         const uint64_t *msg_off, uint64_t n_docs, ymerge_batch_result **res);
int ymerge_updates_v2_batch(ymerge_ctx *ctx, const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_updates,
                            const uint64_t *doc_upd, uint64_t n_docs, ymerge_batch_result **res);
int ydiff_updates_v2_batch(ymerge_ctx *ctx, const uint8_t *bytes, const uint64_t *upd_off, const uint8_t *sv,
                           const uint64_t *sv_off, uint64_t n_docs, ymerge_batch_result **res);
int yencode_state_vector_from_update_v2_batch(ymerge_ctx *ctx, const uint8_t *bytes, const uint64_t *upd_off,
                                              uint64_t n_docs, ymerge_batch_result **res);
int ycompact_updates_v1_batch(ymerge_ctx *ctx, const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_updates,
                              const uint64_t *doc_upd, uint64_t n_docs, ymerge_batch_result **res);
void ymerge_batch_result_destroy(ymerge_batch_result *res);

/* ---------------------------------------------------------------- multi-device (one node)
 * The host-memory merge / diff over n_ctx contexts (one per device, ymerge_ctx_create(dev)).
 * Documents are independent (yrs/src/alt.rs:15-81), so document d is owned by context
 * splitmix64(id) % n_ctx, id = doc_ids[d] (NULL: id = d); every context merges its shard on
 * its own host thread and stream, with no cross-device traffic; *res lists the documents in
 * input order, each byte-identical to the single-context call.  Contexts must not be used by
 * other threads during the call. */
int ymerge_updates_v1_batch_multi(ymerge_ctx *const *ctxs, uint32_t n_ctx, const uint8_t *bytes,
                                  const uint64_t *upd_off, uint64_t n_updates, const uint64_t *doc_upd,
                                  uint64_t n_docs, const uint64_t *doc_ids, ymerge_batch_result **res);
int ydiff_updates_v1_batch_multi(ymerge_ctx *const *ctxs, uint32_t n_ctx, const uint8_t *bytes,
                                 const uint64_t *upd_off, const uint8_t *sv, const uint64_t *sv_off,
                                 uint64_t n_docs, const uint64_t *doc_ids, ymerge_batch_result **res);

#ifdef __cplusplus
}
#endif
#endif
