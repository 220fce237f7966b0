// ysm.h — state-machine walk of one v1 update over the register window (ywin.h).
//
// Same grammar, checks and error order as walk_update + parse_block (ywalk.h,
// ycodec.h; yrs Decode for Update, yrs/src/update.rs:714-749, decode_block :433-488,
// ItemContent::decode yrs/src/block.rs:1786-1835, IdSet::decode id_set.rs:412-426),
// written as ONE loop whose body performs exactly one read (a raw byte for the info
// byte, else one LEB128 u32) followed by a small state switch.  Lanes walking
// differently shaped updates (inserts, deletes, sections, DeleteSets) stay converged
// on the shared read and diverge only in the switch; the code is also a fraction of
// the size of the fully inlined walk.
#pragma once
#include "ywin.h"
#include "ylwin.h"

namespace ym {

enum : uint32_t {
  W_NCL, W_NB, W_CLIENT, W_CLOCK, W_INFO, W_GCLEN, W_OC, W_OK, W_RC, W_RK, W_PI, W_PNAME, W_PC, W_PK, W_PSUB,
  W_CDEL, W_CSTR, W_NDS, W_DCL, W_DNR, W_DST, W_DLN
};

// per-client stored-block counts of one update for the VecDeque::try_reserve check
// (<= 4 distinct clients tracked; see DESIGN.md for the untracked case)
struct SmTrack {
  uint32_t c0, c1, c2, c3, n0, n1, n2, n3, n;
  YM_INLINE uint32_t slot(uint32_t client) {
    uint32_t sl = n > 0 && c0 == client ? 0 : n > 1 && c1 == client ? 1 : n > 2 && c2 == client ? 2
                  : n > 3 && c3 == client ? 3 : 4;
    if (sl == 4 && n < 4) {
      sl = n++;
      if (sl == 0) c0 = client;
      else if (sl == 1) c1 = client;
      else if (sl == 2) c2 = client;
      else c3 = client;
    }
    return sl;
  }
  YM_INLINE uint64_t count(uint32_t sl) const { return sl == 0 ? n0 : sl == 1 ? n1 : sl == 2 ? n2 : sl == 3 ? n3 : 0; }
  YM_INLINE void add(uint32_t sl, uint32_t k) {
    if (sl == 0) n0 += k;
    else if (sl == 1) n1 += k;
    else if (sl == 2) n2 += k;
    else if (sl == 3) n3 += k;
  }
};

// one read of the walk: a raw byte (raw) or a LEB128 u32 with yrs' wrapping_shl (varint.rs:
// 244-260; E_VARINT past 11 bytes); canon = re-encoding gives the same bytes
template <class C> YM_INLINE int wc_read(C &c, bool raw, uint32_t &v, bool &canon) {
  uint32_t sh = 0, nbytes = 0, b = 0;
  v = 0;
  for (;;) {
    if (c.i >= c.n) return E_EOS;
    b = wc_byte(c, c.i++);
    if (raw) {
      v = b;
      return 0;
    }
    v |= (b & 0x7f) << (sh & 31);
    sh += 7;
    nbytes++;
    if (b < 0x80) break;
    if (sh > 70) return E_VARINT;
  }
  canon = nbytes == varlen(v) && (nbytes != 5 || b < 16);
  return 0;
}
// OR of the bytes [s0, s0 + n) (the ASCII test of a string)
template <class C> YM_INLINE uint32_t wc_or(C &c, uint32_t s0, uint32_t n) {
  uint32_t hi = 0;
  for (uint32_t q = 0; q < n; q++) hi |= wc_byte(c, s0 + q);
  return hi;
}

// Content refs 3 (Binary), 7 (Type, not weak) and 8 (Any of scalars and strings), restated
// inline on the cursor (ItemContent::decode, yrs/src/block.rs:1786-1835; Any::decode,
// yrs/src/any.rs:37-83; TypeRef::decode, yrs/src/types/mod.rs:160-200): the out-of-line
// parse_content_slow costs a call (register saves to scratch) per block, which dominated walks
// of rich documents.  Returns 1 (parsed: bi.len / bi.reenc set, cursor past the content), 0
// (not this shape: cursor restored, parse_content_slow takes it) or an error in read order.
template <class C> YM_INLINE int sm_content_inline(C &c, uint32_t ref, BlockInfo &bi) {
  const uint32_t c0 = c.i;
  uint32_t v = 0;
  bool canon = true;
  if (ref == 3) {
    YM_TRY(wc_read(c, false, v, canon));
    bi.reenc |= !canon;
    YM_TRY(wc_skip(c, v));
    bi.len = 1;
    return 1;
  }
  if (ref == 7) {
    YM_TRY(wc_read(c, true, v, canon));
    if (v == 7) { // weak link: parse_content_slow
      c.i = c0;
      return 0;
    }
    bi.len = 1;
    if (v == 3) {
      YM_TRY(wc_read(c, false, v, canon));
      bi.reenc |= !canon;
      return wc_skip(c, v) ? E_EOS : 1;
    }
    if (v <= 6 || v == 9 || v == 15) return 1;
    return E_UNEXPECTED;
  }
  if (ref != 8) return 0;
  uint32_t n;
  YM_TRY(wc_read(c, false, n, canon));
  if ((uint64_t)n * 24 > ALLOC_LIMIT) {
    c.i = c0;
    return 0;
  }
  bool reenc = !canon;
  for (uint32_t k = 0; k < n; k++) {
    uint32_t tag;
    YM_TRY(wc_read(c, true, tag, canon));
    switch (tag) {
    case 127: case 126: case 121: case 120: break;
    case 125: { // signed varint (varint.rs:262-281), canonical iff num_encode gives the same bytes
      const uint32_t s0 = c.i;
      uint32_t b = 0;
      if (c.i >= c.n) return E_EOS;
      b = wc_byte(c, c.i++);
      uint64_t num = b & 0x3f;
      uint32_t len = 6;
      const bool neg = (b & 0x40) != 0;
      if (b & 0x80) {
        for (;;) {
          if (c.i >= c.n) return E_EOS;
          b = wc_byte(c, c.i++);
          num |= (uint64_t)(b & 0x7f) << (len & 63);
          len += 7;
          if (b < 0x80) break;
          if (len > 70) return E_VARINT;
        }
      }
      const int64_t iv = neg ? (int64_t)(0 - num) : (int64_t)num;
      struct Cmp {
        C &cur;
        uint32_t at, end;
        bool eq;
        __device__ void u8(uint8_t x) {
          if (at >= end || wc_byte(cur, at) != x) eq = false;
          at++;
        }
        __device__ void bytes(const uint8_t *, uint32_t) {}
      } cmp{c, s0 - 1, c.i, true};
      num_encode(cmp, i64_to_f64_bits(iv));
      if (!cmp.eq || cmp.at != cmp.end) reenc = true;
      break;
    }
    case 124: { // f32: canonical unless NaN or integral-safe
      if (c.n - c.i < 4) return E_EOS;
      uint32_t fb = 0;
      for (uint32_t q = 0; q < 4; q++) fb = fb << 8 | wc_byte(c, c.i + q);
      c.i += 4;
      const uint32_t ex = (fb >> 23) & 0xFF;
      struct Peek {
        uint8_t first = 0;
        bool any = false;
        __device__ void u8(uint8_t x) {
          if (!any) first = x;
          any = true;
        }
        __device__ void bytes(const uint8_t *, uint32_t) {}
      } pk;
      num_encode(pk, f32_to_f64_bits(fb));
      if ((ex == 0xFF && (fb & 0x7FFFFF)) || pk.first == 125) reenc = true;
      break;
    }
    case 123: { // f64: canonical iff it stays tag 123
      if (c.n - c.i < 8) return E_EOS;
      uint64_t bits = 0;
      for (uint32_t q = 0; q < 8; q++) bits = bits << 8 | wc_byte(c, c.i + q);
      c.i += 8;
      struct Peek {
        uint8_t first = 0;
        bool any = false;
        __device__ void u8(uint8_t x) {
          if (!any) first = x;
          any = true;
        }
        __device__ void bytes(const uint8_t *, uint32_t) {}
      } pk;
      num_encode(pk, bits);
      if (pk.first != 123) reenc = true;
      break;
    }
    case 122:
      if (c.n - c.i < 8) return E_EOS;
      c.i += 8;
      break;
    case 119: case 116:
      YM_TRY(wc_read(c, false, v, canon));
      if (!canon) reenc = true;
      YM_TRY(wc_skip(c, v));
      break;
    case 118: case 117: // maps / arrays: parse_content_slow from the content's start
      c.i = c0;
      return 0;
    default: return E_UNEXPECTED;
    }
  }
  bi.len = n;
  bi.reenc |= reenc;
  return 1;
}

#ifndef YM_SM_PROBE
#define YM_SM_PROBE(st) // (tools/walkbench.hip: per-state cycle histogram)
#endif
template <class S, class C> YM_INLINE int smwalk_update(C &c, S &s) {
  uint32_t st = W_NCL;
  uint32_t ncl = 0, isec = 0, nb = 0, client = 0, clock = 0, j = 0, stored = 0, slot = 4;
  uint32_t nds = 0, ids = 0, dclient = 0, nr = 0, kr = 0, rst = 0;
  uint32_t info = 0, want = 0, bpos = 0;
  BlockInfo bi;
  bi.kind = BK_ITEM;
  bi.ref = 0;
  bi.info = 0;
  bi.reenc = bi.unsupported = bi.enc_panic = false;
  bi.len = 0;
  bi.canon = 0;
  SmTrack tc{0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (;;) {
    YM_SM_PROBE(st);
    // ---- the one read of this step
    uint32_t v = 0;
    bool canon = true;
    {
      const bool raw = st == W_INFO;
      if (raw) {
        bpos = c.i;
        wc_ensure(c, 48); // the whole block in the window: one wait per block
      } else if (st == W_DST) {
        wc_ensure(c, 20);
      }
      YM_TRY(wc_read(c, raw, v, canon));
    }
    // ---- state transition
    bool block_end = false, header_end = false;
    switch (st) {
    case W_NCL:
      ncl = v;
      if (ncl && cap_to_buckets(ncl) * 41ull > ALLOC_LIMIT) return E_NEM; // try_reserve
      st = ncl ? W_NB : W_NDS;
      break;
    case W_NB: nb = v; st = W_CLIENT; break;
    case W_CLIENT: client = v; st = W_CLOCK; break;
    case W_CLOCK:
      clock = v;
      slot = ncl > 1 ? tc.slot(client) : 4;
      if ((tc.count(slot) + nb) * 32ull > ALLOC_LIMIT) return E_NEM; // VecDeque::try_reserve
      s.on_section(client);
      stored = 0;
      j = 0;
      if (nb) {
        st = W_INFO;
      } else {
        isec++;
        st = isec < ncl ? W_NB : W_NDS;
      }
      break;
    case W_INFO:
      info = v;
      bi.info = (uint8_t)info;
      bi.reenc = bi.unsupported = bi.enc_panic = false;
      if (info == 10 || info == 0) {
        bi.kind = info == 10 ? BK_SKIP : BK_GC;
        bi.ref = 0;
        st = W_GCLEN;
      } else {
        bi.kind = BK_ITEM;
        want = info & 0xCF; // 0x10 never re-emitted; 0x20 only when parent_sub decoded
        st = (info & 0x80) ? W_OC : (info & 0x40) ? W_RC : W_PI;
      }
      break;
    case W_GCLEN:
      bi.len = v;
      bi.reenc = !canon;
      block_end = true;
      break;
    case W_OC: bi.reenc |= !canon; st = W_OK; break;
    case W_OK:
      bi.reenc |= !canon;
      if (info & 0x40) st = W_RC;
      else if ((info & 0xC0) == 0) st = W_PI;
      else header_end = true;
      break;
    case W_RC: bi.reenc |= !canon; st = W_RK; break;
    case W_RK:
      bi.reenc |= !canon;
      if ((info & 0xC0) == 0) st = W_PI;
      else header_end = true;
      break;
    case W_PI:
      bi.reenc |= !canon || (v != 1 && v != 0);
      st = v == 1 ? W_PNAME : W_PC;
      break;
    case W_PNAME:
    case W_PSUB:
      bi.reenc |= !canon;
      YM_TRY(wc_skip(c, v));
      if (st == W_PSUB) {
        want |= 0x20;
        header_end = true;
      } else if (info & 0x20) {
        st = W_PSUB;
      } else {
        header_end = true;
      }
      break;
    case W_PC: bi.reenc |= !canon; st = W_PK; break;
    case W_PK:
      bi.reenc |= !canon;
      if (info & 0x20) st = W_PSUB;
      else header_end = true;
      break;
    case W_CDEL:
      bi.len = v;
      bi.reenc |= !canon;
      block_end = true;
      break;
    case W_CSTR: {
      bi.reenc |= !canon;
      const uint32_t s0 = c.i;
      YM_TRY(wc_skip(c, v));
      block_end = true;
      if (v == 1) {
        bi.len = 1;
        break;
      }
      const uint32_t hi = wc_or(c, s0, v);
      if (hi < 0x80) {
        bi.len = v;
        break;
      }
      const uint8_t *sp = c.p + s0; // non-ASCII: UTF-16 length on the plain pointer (cold)
      str_info16(sp, v, bi);
      break;
    }
    case W_NDS:
      nds = v;
      YM_TRY(s.on_ds_begin(nds));
      ids = 0;
      if (!nds) return s.on_ds_done();
      st = W_DCL;
      break;
    case W_DCL: dclient = v; st = W_DNR; break;
    case W_DNR:
      nr = v;
      YM_TRY(s.on_ds_entry(dclient, nr));
      kr = 0;
      if (nr) {
        st = W_DST;
      } else {
        if (++ids == nds) return s.on_ds_done();
        st = W_DCL;
      }
      break;
    case W_DST: rst = v; st = W_DLN; break;
    case W_DLN:
      if ((uint64_t)rst + v > 0xFFFFFFFFull) return E_PANIC;
      s.on_ds_range(rst, rst + v);
      if (++kr < nr) {
        st = W_DST;
      } else {
        if (++ids == nds) return s.on_ds_done();
        st = W_DCL;
      }
      break;
    default: return E_OTHER;
    }
    if (header_end) {
      if (want != info) bi.reenc = true;
      const uint32_t ref = info & 15;
      bi.ref = (uint8_t)ref;
      if (ref == 1) {
        st = W_CDEL;
      } else if (ref == 4) {
        st = W_CSTR;
      } else {
        const int hr = sm_content_inline(c, ref, bi);
        if (hr > 1) return hr; // (an error code)
        if (hr == 0) { // cold content kinds: out of line, on the plain pointer
          SlowRes r = parse_content_slow(c.p, c.n, c.i, (uint8_t)ref, bi.reenc);
          if (r.err) return r.err;
          c.i = r.pos;
          bi.len = r.len;
          bi.reenc = r.reenc;
          bi.unsupported = r.unsupported;
        }
        block_end = true;
      }
    }
    if (block_end) {
      if (!(bi.kind == BK_ITEM && bi.len == 0)) { // Item::new -> None: dropped
        if ((uint64_t)clock + bi.len > 0xFFFFFFFFull) return E_PANIC;
        YM_TRY(s.on_block(client, clock, bi, bpos, c.i - bpos));
        stored++;
        clock += bi.len;
      }
      if (++j < nb) {
        st = W_INFO;
      } else {
        tc.add(slot, stored);
        isec++;
        st = isec < ncl ? W_NB : W_NDS;
      }
    }
  }
}

// byte copy global -> global through the register window: each 32-byte window is
// loaded once ahead of its stores (a plain byte loop serialises the load latency per
// byte: the compiler cannot hoist a load above a possibly aliasing store)
YM_INLINE void copy_window(uint8_t *dst, const uint8_t *src, uint32_t len) {
  WCur c;
  wc_init(c, src, len);
  for (uint32_t q = 0; q < len; q++) dst[q] = (uint8_t)wc_byte(c, q);
}
// byte copy global -> (LDS stage or global) in groups of 16: the 16 byte loads of a group
// are issued before any store (one memory latency per group), one instruction per byte
// each way instead of the window's select tree per byte
// Copies len bytes, 16 at a time: the (<= 5) aligned source dwords covering each 16-byte
// piece are loaded together and realigned with alignbyte (5 loads instead of 16 byte loads
// per piece); the destination is written bytewise (any alignment).  The source arena is
// dword-aligned, so the covering dwords stay inside it.
YM_INLINE void copy_bytes16(uint8_t *dst, const uint8_t *src, uint32_t len) {
  const uint32_t mis = (uint32_t)((uintptr_t)src & 3);
  const uint32_t *s4 = (const uint32_t *)(src - mis);
  for (uint32_t q0 = 0; q0 < len; q0 += 16) {
    const uint32_t need = mis + len - q0; // bytes from the first covering dword on
    uint32_t w[5];
#pragma unroll
    for (uint32_t k = 0; k < 5; k++) w[k] = 4 * k < need ? s4[(q0 >> 2) + k] : 0u;
    uint32_t o[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) o[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], mis);
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
      if (q0 + k < len) dst[q0 + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
  }
}
YM_INLINE bool equal_window(const uint8_t *a, const uint8_t *b, uint32_t len) {
  WCur x, y;
  wc_init(x, a, len);
  wc_init(y, b, len);
  uint32_t diff = 0;
  for (uint32_t q = 0; q < len && !diff; q++) diff = wc_byte(x, q) ^ wc_byte(y, q);
  return diff == 0;
}

} // namespace ym
