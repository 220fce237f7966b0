// CPU build of ycompact.hip's per-document body (compact_doc) over an arena batch, for the
// CPU parity tests against the oracle (test tooling, see hip/hip_runtime.h here).
#include "../../y-crdt_amd/csrc/ycompact.hip"
#include <vector>

extern "C" void emu_compact_batch(const uint8_t *bytes, const uint64_t *upd_off, const uint64_t *doc_upd,
                                  uint32_t n_docs, uint8_t *out, uint64_t *out_start, uint64_t *out_len,
                                  uint8_t *status, uint8_t *why) {
  ym::BatchIn b{bytes, upd_off, doc_upd, n_docs, nullptr, nullptr};
  ym::FastOut o{out, out_start, out_len, status, why, nullptr, nullptr, nullptr};
  ym::ym_set_grammar(0);
  std::vector<uint32_t> hdr((size_t)n_docs * ym::CP_HDR + 1);
  std::vector<uint64_t> need(n_docs + 1), off(n_docs + 1, 0);
  alignas(16) uint8_t cstage[ym::CP_STAGE];
  for (uint32_t d = 0; d < n_docs; d++) ym::compact_count_doc(b, hdr.data(), need.data(), d, cstage);
  for (uint32_t d = 0; d < n_docs; d++) off[d + 1] = off[d] + need[d];
  std::vector<uint32_t> scr(off[n_docs] + 16);
  alignas(16) uint8_t stage[ym::CP_STAGE];
  uint32_t misc[ym::M_END];
  for (uint32_t d = 0; d < n_docs; d++) ym::compact_doc(b, o, hdr.data(), off.data(), scr.data(), d, stage, misc);
}
