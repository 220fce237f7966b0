// CPU build of the string / JSON helpers of ycodec.h and yjson.h, for the CPU tests that pin the
// fast paths against the general walks (tests/test_codec_emu.py; test tooling, see
// hip/hip_runtime.h here).  Callers pass buffers with >= 16 readable bytes on both sides of the
// string: the fast paths load whole aligned 16-byte chunks, as they do in the padded device arena.
#include "hip/hip_runtime.h"
#include "../../y-crdt_amd/csrc/ycodec.h"

namespace {
struct Buf {
  uint8_t *p;
  uint64_t n, cap;
  void u8(uint8_t b) {
    if (n < cap) p[n] = b;
    n++;
  }
  void bytes(const uint8_t *s, uint32_t k) {
    for (uint32_t i = 0; i < k; i++) u8(s[i]);
  }
};
} // namespace

// str_info16 (the product path: SWAR fast path for >= 64 bytes, else the serial walk): out =
// UTF-16 length, re-encode flag, panic flag
extern "C" void emu_str_info16(const uint8_t *s, uint32_t n, uint32_t *out) {
  ym::BlockInfo bi{};
  ym::str_info16(s, n, bi);
  out[0] = bi.len;
  out[1] = bi.reenc;
  out[2] = bi.enc_panic;
}
// the same three values from the serial walk only (utf8_next over every char, then split16)
extern "C" void emu_str_serial(const uint8_t *s, uint32_t n, uint32_t *out) {
  uint32_t k = 0, i = 0;
  while (i < n) k += ym::ch_len16(ym::utf8_next(s, n, i));
  if (n == 1) k = 1; // SplittableString::len: a one-byte string is 1 whatever the kind (block.rs:1391-1395)
  out[0] = k;
  out[1] = out[2] = 0;
  if (k > 1) {
    uint32_t bo;
    if (ym::str_split16(s, n, k, bo)) out[2] = 1;
    else if (bo != n) out[1] = 1;
  }
}
// str_fast16 alone: 1 = accepted (len in *len), 0 = left to the serial walk
extern "C" int emu_str_fast16(const uint8_t *s, uint32_t n, uint32_t *len) { return ym::str_fast16(s, n, *len) ? 1 : 0; }
extern "C" int emu_bytes_ascii(const uint8_t *s, uint32_t n) { return ym::bytes_ascii(s, n) ? 1 : 0; }
extern "C" int emu_json_plain(const uint8_t *s, uint32_t n) { return ym::json_plain(s, n) ? 1 : 0; }
// json_canon (mode 0, with the shortcut) or json_canon_walk (mode 1): bytes written (may exceed
// cap: then only cap were stored), or -1 on E_JSON
extern "C" int64_t emu_json(const uint8_t *s, uint32_t n, int mode, uint8_t *out, uint64_t cap) {
  Buf w{out, 0, cap};
  const int rc = mode ? ym::json_canon_walk(s, n, w) : ym::json_canon(s, n, w);
  return rc ? -1 : (int64_t)w.n;
}
