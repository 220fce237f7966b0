// ywin.h — register-window reader for lane-serial walks over HBM-resident updates.
//
// A lane that walks a whole (large) update byte by byte cannot afford one memory
// round trip per byte.  WCur keeps a 32-byte window of the stream in eight VGPRs,
// loaded with two 16-byte aligned vector loads, and serves bytes out of it with a
// select tree (no dynamic register indexing, no scratch).  A window load never
// touches a 16-byte chunk that holds no valid byte of the stream, so it cannot
// cross into an unmapped page.
//
// wparse_block restates parse_block (ycodec.h; yrs Update::decode_block,
// yrs/src/update.rs:433-488 + ItemContent::decode, yrs/src/block.rs:1786-1835) on
// the window for the hot content kinds (GC, Skip, Deleted, String); the cold kinds
// go through parse_content_slow on the plain global pointer.
#pragma once
#include "ycodec.h"

namespace ym {

struct WCur {
  const uint8_t *p; // stream start (global memory)
  uint32_t n, i;    // length, position
  uint64_t wa;      // absolute address of the window ([wa, wa + 32))
  uint32_t w0, w1, w2, w3, w4, w5, w6, w7;
};

YM_INLINE void wc_init(WCur &c, const uint8_t *p, uint32_t n) {
  c.p = p;
  c.n = n;
  c.i = 0;
  c.wa = ~0ull << 8; // forces a load on first access
  c.w0 = c.w1 = c.w2 = c.w3 = c.w4 = c.w5 = c.w6 = c.w7 = 0;
}

YM_INLINE void wc_load(WCur &c, uint64_t a) { // a: 16-byte aligned, holds a valid byte
  const uint4 *q = (const uint4 *)a;
  uint4 x = q[0];
  c.w0 = x.x;
  c.w1 = x.y;
  c.w2 = x.z;
  c.w3 = x.w;
  if (a + 16 < (uint64_t)(c.p + c.n)) {
    uint4 y = q[1];
    c.w4 = y.x;
    c.w5 = y.y;
    c.w6 = y.z;
    c.w7 = y.w;
  }
  c.wa = a;
}

// byte at stream position pos (< n)
YM_INLINE uint32_t wc_byte(WCur &c, uint32_t pos) {
  uint64_t a = (uint64_t)(c.p + pos);
  uint64_t off = a - c.wa;
  if (off >= 32) {
    wc_load(c, a & ~15ull);
    off = a & 15;
  }
  const uint32_t k = (uint32_t)off >> 2;
  const uint32_t lo = (k & 1) ? ((k & 2) ? c.w3 : c.w1) : ((k & 2) ? c.w2 : c.w0);
  const uint32_t hi = (k & 1) ? ((k & 2) ? c.w7 : c.w5) : ((k & 2) ? c.w6 : c.w4);
  const uint32_t d = (k & 4) ? hi : lo;
  return (d >> (((uint32_t)off & 3) * 8)) & 0xFF;
}

YM_INLINE int wc_u8(WCur &c, uint8_t &v) {
  if (c.i >= c.n) return E_EOS;
  v = (uint8_t)wc_byte(c, c.i++);
  return 0;
}
YM_INLINE int wc_skip(WCur &c, uint64_t len) {
  if (len > (uint64_t)(c.n - c.i)) return E_EOS;
  c.i += (uint32_t)len;
  return 0;
}
// read_var_u32 (varint.rs:244-260, wrapping_shl quirk); canon = re-encoding gives the same bytes
YM_INLINE int wc_var_u32(WCur &c, uint32_t &v, bool &canon) {
  uint32_t num = 0, len = 0, nb = 0;
  uint8_t b = 0;
  for (;;) {
    YM_TRY(wc_u8(c, b));
    num |= (uint32_t)(b & 0x7f) << (len & 31);
    len += 7;
    nb++;
    if (b < 0x80) break;
    if (len > 70) return E_VARINT;
  }
  v = num;
  canon = nb == varlen(num) && (nb != 5 || b < 16);
  return 0;
}
YM_INLINE int wc_var_u64(WCur &c, uint64_t &v, bool &canon) {
  uint64_t num = 0;
  uint32_t len = 0, nb = 0;
  uint8_t b = 0;
  for (;;) {
    YM_TRY(wc_u8(c, b));
    num |= (uint64_t)(b & 0x7f) << (len & 63);
    len += 7;
    nb++;
    if (b < 0x80) break;
    if (len > 70) return E_VARINT;
  }
  v = num;
  canon = nb == varlen(num) && (nb != 10 || b < 2);
  return 0;
}

// parse_block (ycodec.h) on the window; identical results, including error order
YM_INLINE int wparse_block(WCur &c, BlockInfo &bi) {
  uint8_t info;
  bool cn;
  YM_TRY(wc_u8(c, info));
  bi.info = info;
  bi.reenc = false;
  bi.unsupported = false;
  bi.enc_panic = false;
  if (info == 10 || info == 0) {
    bi.kind = info == 10 ? BK_SKIP : BK_GC;
    bi.ref = 0;
    YM_TRY(wc_var_u32(c, bi.len, cn));
    bi.reenc = !cn;
    return 0;
  }
  bi.kind = BK_ITEM;
  const bool cant_copy = (info & 0xC0) == 0;
  uint32_t v;
  uint8_t want = info & 0xCF;
  if (info & 0x80) {
    YM_TRY(wc_var_u32(c, v, cn));
    bi.reenc |= !cn;
    YM_TRY(wc_var_u32(c, v, cn));
    bi.reenc |= !cn;
  }
  if (info & 0x40) {
    YM_TRY(wc_var_u32(c, v, cn));
    bi.reenc |= !cn;
    YM_TRY(wc_var_u32(c, v, cn));
    bi.reenc |= !cn;
  }
  if (cant_copy) {
    uint32_t pi;
    YM_TRY(wc_var_u32(c, pi, cn));
    bi.reenc |= !cn || (pi != 1 && pi != 0);
    if (pi == 1) {
      YM_TRY(wc_var_u32(c, v, cn));
      bi.reenc |= !cn;
      YM_TRY(wc_skip(c, v));
    } else {
      YM_TRY(wc_var_u32(c, v, cn));
      bi.reenc |= !cn;
      YM_TRY(wc_var_u32(c, v, cn));
      bi.reenc |= !cn;
    }
    if (info & 0x20) {
      want |= 0x20;
      YM_TRY(wc_var_u32(c, v, cn));
      bi.reenc |= !cn;
      YM_TRY(wc_skip(c, v));
    }
  }
  if (want != info) bi.reenc = true;
  const uint8_t ref = info & 15;
  bi.ref = ref;
  if (ref == 1) {
    YM_TRY(wc_var_u32(c, bi.len, cn));
    bi.reenc |= !cn;
    return 0;
  }
  if (ref == 4) {
    YM_TRY(wc_var_u32(c, v, cn));
    bi.reenc |= !cn;
    const uint32_t s0 = c.i;
    YM_TRY(wc_skip(c, v));
    if (v == 1) {
      bi.len = 1;
      return 0;
    }
    uint32_t hi = 0;
    for (uint32_t q = 0; q < v; q++) hi |= wc_byte(c, s0 + q);
    if (hi < 0x80) {
      bi.len = v;
      return 0;
    }
    const uint8_t *s = c.p + s0; // non-ASCII: UTF-16 length on the plain pointer (cold)
    bi.len = str_len16(s, v);
    if (bi.len > 1) {
      uint32_t bo;
      if (str_split16(s, v, bi.len, bo)) bi.enc_panic = true;
      else if (bo != v) bi.reenc = true;
    }
    return 0;
  }
  SlowRes r = parse_content_slow(c.p, c.n, c.i, ref, bi.reenc);
  if (r.err) return r.err;
  c.i = r.pos;
  bi.len = r.len;
  bi.reenc = r.reenc;
  bi.unsupported = r.unsupported;
  return 0;
}

} // namespace ym
