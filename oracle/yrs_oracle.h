/*
 * yrs_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the yrs 0.19.2 binary-update algebra over lib0 v1 bytes
 * (reference: yrs/src/alt.rs:15-81, yrs/src/update.rs:107-749).  It is the
 * parity checker for the HIP engine in y-crdt_amd/ and the "port" CPU
 * baseline of bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product path never does.
 *
 * Parity pin: the four byte-exact KATs of yrs/src/alt.rs:103-160, the v1
 * payloads of yrs/src/tests/compatibility_tests.rs and yrs/src/update.rs:1097,
 * plus fixtures produced by the offline Yjs bundle (tests/golden/).
 */
#ifndef YRS_ORACLE_H
#define YRS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: 0..9 mirror yffi's error codes (yffi/src/lib.rs:1137-1174) */
enum {
  YO_OK = 0,
  YO_ERR_VAR_INT = 2,
  YO_ERR_EOS = 3,
  YO_ERR_UNEXPECTED_VALUE = 4,
  YO_ERR_INVALID_JSON = 5,
  YO_ERR_OTHER = 6,
  YO_ERR_NOT_ENOUGH_MEMORY = 7,
  YO_ERR_REFERENCE_PANIC = 20, /* yrs itself would panic/abort on this input */
  YO_ERR_UNSUPPORTED = 21      /* Embed/Format JSON round trip: not restated yet */
};

/* mode for merge: 0 = literal reference loop (per-iteration stable insertion
 * sort of all live decoders, DS re-squash after every input — same complexity
 * as yrs), 1 = equivalent fast form (decoder heap, single final squash). */
/* store-based compaction: a Doc (GC on) applies the updates in order, one transaction each, then
 * encode_state_as_update_v1 (yrs_oracle_store.c) */
int yo_compact_updates_v1(const uint8_t *const *updates, const size_t *lens, size_t n, uint8_t **out,
                          size_t *out_len);
int yo_merge_updates_v1(const uint8_t *const *updates, const size_t *lens, size_t n,
                        int mode, uint8_t **out, size_t *out_len);
int yo_diff_updates_v1(const uint8_t *update, size_t update_len, const uint8_t *sv,
                       size_t sv_len, uint8_t **out, size_t *out_len);
int yo_encode_state_vector_from_update_v1(const uint8_t *update, size_t len, uint8_t **out,
                                          size_t *out_len);
void yo_free(void *p);
/* lib0 v2 (yrs/src/alt.rs:35-48, 63-66, 88-97; codec yrs/src/updates/{decoder,encoder}.rs) */
int yo_merge_updates_v2(const uint8_t *const *updates, const size_t *lens, size_t n, int mode, uint8_t **out,
                        size_t *out_len);
int yo_diff_updates_v2(const uint8_t *update, size_t update_len, const uint8_t *sv, size_t sv_len, uint8_t **out,
                       size_t *out_len);
int yo_encode_state_vector_from_update_v2(const uint8_t *update, size_t len, uint8_t **out, size_t *out_len);
int yo_merge_updates_v1_to_v2(const uint8_t *const *updates, const size_t *lens, size_t n, int mode, uint8_t **out,
                              size_t *out_len);
int yo_convert_update_v1_to_v2(const uint8_t *update, size_t len, uint8_t **out, size_t *out_len);
int yo_convert_update_v2_to_v1(const uint8_t *update, size_t len, uint8_t **out, size_t *out_len);
/* y-sync (yrs/src/sync/protocol.rs:62-69, 219-272): SyncStep1 message of an update's state
 * vector, and the SyncStep2 reply to a client's SyncStep1 message */
int yo_sync_step1_v1(const uint8_t *update, size_t len, uint8_t **out, size_t *out_len);
int yo_sync_step2_v1(const uint8_t *update, size_t len, const uint8_t *msg, size_t mlen, uint8_t **out,
                     size_t *out_len);
int yo_sv_roundtrip(const uint8_t *p, size_t n, uint8_t **out, size_t *out_len);
int yo_ds_offset(const uint8_t *p, size_t n, size_t *off);

/* Batched merge over an arena: doc d owns updates [doc_upd[d], doc_upd[d+1]),
 * update u owns bytes [upd_off[u], upd_off[u+1]).  Outputs are written to a
 * malloc'd arena (*out, out_off[n_docs+1]) and status[n_docs].  `threads`
 * worker threads split the docs (0 = 1 thread). */
int yo_merge_batch(const uint8_t *bytes, const uint64_t *upd_off, const uint64_t *doc_upd,
                   size_t n_docs, int mode, int threads, uint8_t **out, uint64_t *out_off,
                   uint8_t *status);
int yo_diff_batch(const uint8_t *ubytes, const uint64_t *u_off, const uint8_t *svbytes,
                  const uint64_t *sv_off, size_t n_docs, int threads, uint8_t **out,
                  uint64_t *out_off, uint8_t *status);

int yo_sv_batch(const uint8_t *ubytes, const uint64_t *u_off, size_t n_docs, int threads, uint8_t **out,
                uint64_t *out_off, uint8_t *status);

#ifdef __cplusplus
}
#endif
#endif
