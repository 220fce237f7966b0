// ycodec.h — device-side lib0 v1 codec for the MI355X update-compaction engine.
//
// Restates (for gfx950 device code) the decode/encode rules the engine must be
// bit-exact with:
//   varints            yrs/src/encoding/varint.rs:184-281 (u32 wrapping_shl quirk)
//   block decode       yrs/src/update.rs:433-488, content block.rs:1786-1835
//   block encode       yrs/src/slice.rs:199-251, block.rs:1711-1754, info block.rs:1363-1369
//   Any                yrs/src/any.rs:37-183 (number canonicalisation any.rs:136-154)
//   TypeRef / Move / Doc options  types/mod.rs:118-200, moving.rs:277-333, doc.rs:814-872
//   hashbrown order    std HashMap + ClientHasher (utils/client_hasher.rs)
//   Embed/Format JSON  serde_json + ryu round trip (yjson.h)
// Policies shared with the CPU oracle: allocation limit 2^36 B, Any
// nesting <= 64 (UNSUPPORTED beyond), Any/JSON maps with duplicate keys collapse to the
// last value, written at the position of the key's last occurrence.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ym {

enum : int {
  S_OK = 0,
  E_VARINT = 2,
  E_EOS = 3,
  E_UNEXPECTED = 4,
  E_JSON = 5,
  E_OTHER = 6,
  E_NEM = 7,
  E_PANIC = 20,
  E_UNSUPPORTED = 21,
};
constexpr uint64_t ALLOC_LIMIT = 1ull << 36;
constexpr int ANY_MAX_DEPTH = 64;

#define YM_INLINE __device__ __attribute__((always_inline)) inline
#define YM_TRY(x)                                                                                  \
  do {                                                                                             \
    int _e = (x);                                                                                  \
    if (_e) return _e;                                                                             \
  } while (0)

// ------------------------------------------------------------------ cursor
struct Cur {
  const uint8_t *p;
  uint32_t n, i;
};
__device__ __forceinline__ int rd_u8(Cur &c, uint8_t &v) {
  if (c.i >= c.n) return E_EOS;
  v = c.p[c.i++];
  return 0;
}
__device__ __forceinline__ int rd_skip(Cur &c, uint64_t len) {
  if (len > (uint64_t)(c.n - c.i)) return E_EOS;
  c.i += (uint32_t)len;
  return 0;
}
__device__ __forceinline__ uint32_t varlen(uint64_t v) {
  uint32_t k = 1;
  while (v >= 0x80) {
    v >>= 7;
    k++;
  }
  return k;
}
// read_var_u32 (varint.rs:244-260); *canon = re-encoding gives the same bytes
__device__ __forceinline__ int rd_var_u32(Cur &c, uint32_t &v, bool &canon) {
  uint32_t num = 0, len = 0, nb = 0;
  uint8_t b = 0;
  for (;;) {
    YM_TRY(rd_u8(c, b));
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
__device__ __forceinline__ int rd_var_u64(Cur &c, uint64_t &v, bool &canon) {
  uint64_t num = 0;
  uint32_t len = 0, nb = 0;
  uint8_t b = 0;
  for (;;) {
    YM_TRY(rd_u8(c, b));
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
// read_var_i64 (varint.rs:262-281)
__device__ __forceinline__ int rd_var_i64(Cur &c, int64_t &v) {
  uint8_t b;
  YM_TRY(rd_u8(c, b));
  uint64_t num = b & 0x3f;
  uint32_t len = 6;
  bool neg = (b & 0x40) != 0;
  if (b & 0x80) {
    for (;;) {
      YM_TRY(rd_u8(c, b));
      num |= (uint64_t)(b & 0x7f) << (len & 63);
      len += 7;
      if (b < 0x80) break;
      if (len > 70) return E_VARINT;
    }
  }
  v = neg ? (int64_t)(0 - num) : (int64_t)num;
  return 0;
}

// ------------------------------------------------------------------ writers
struct Counter {
  uint64_t n = 0;
  __device__ __forceinline__ void u8(uint8_t) { n++; }
  __device__ __forceinline__ void bytes(const uint8_t *, uint32_t k) { n += k; }
};
struct Writer {
  uint8_t *p;
  uint64_t n;
  __device__ __forceinline__ void u8(uint8_t b) { p[n++] = b; }
  // in groups of 16 whose loads are all issued before the group's stores (a plain byte loop
  // waits one load latency per byte: the stores may alias the next loads)
  __device__ __forceinline__ void bytes(const uint8_t *s, uint32_t k) {
    uint32_t i = 0;
    for (; i + 16 <= k; i += 16) {
      uint8_t t[16];
#pragma unroll
      for (uint32_t j = 0; j < 16; j++) t[j] = s[i + j];
#pragma unroll
      for (uint32_t j = 0; j < 16; j++) p[n + i + j] = t[j];
    }
    for (; i < k; i++) p[n + i] = s[i];
    n += k;
  }
};
// no byte >= 0x80 in s[0, n): 16-byte aligned vector loads, 128 bytes in flight per step (the
// aligned chunks covering s[0, n) stay inside the padded arena); a lane checking a 100 KB
// pasted string byte by byte held k_lp_expand for 17 ms on the editing traces
__device__ __forceinline__ bool bytes_ascii(const uint8_t *s, uint32_t n) {
  if (n == 0) return true;
  const uint64_t lo = (uint64_t)s, hi = lo + n;
  for (uint64_t a = lo & ~15ull; a < hi; a += 128) {
    uint4 x[8];
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (a + 16 * k < hi) x[k] = *(const uint4 *)(a + 16 * k);
    uint32_t orw = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (a + 16 * k >= hi) break;
      const uint32_t w[4] = {x[k].x, x[k].y, x[k].z, x[k].w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint64_t wb = a + 16 * k + 4 * j;
        uint32_t m = 0x80808080u;
        if (wb < lo) m = lo - wb >= 4 ? 0u : m & (~0u << (8 * (uint32_t)(lo - wb)));
        if (wb + 4 > hi) m = hi <= wb ? 0u : m & ((1u << (8 * (uint32_t)(hi - wb))) - 1u);
        orw |= w[j] & m;
      }
    }
    if (orw) return false;
  }
  return true;
}
template <class W> __device__ __forceinline__ void w_var(W &w, uint64_t v) {
  while (v >= 0x80) {
    w.u8((uint8_t)(v | 0x80));
    v >>= 7;
  }
  w.u8((uint8_t)v);
}
template <class W> __device__ __forceinline__ void w_var_i64(W &w, int64_t value) {
  bool neg = value < 0;
  if (neg) value = (int64_t)(0 - (uint64_t)value);
  w.u8((uint8_t)((value > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (uint8_t)(63 & value)));
  value >>= 6;
  while (value > 0) {
    w.u8((uint8_t)((value > 127 ? 0x80 : 0) | (uint8_t)(127 & value)));
    value >>= 7;
  }
}
template <class W> __device__ __forceinline__ void w_str(W &w, const uint8_t *s, uint32_t n) {
  w_var(w, n);
  w.bytes(s, n);
}

#include "yjson.h"

// ------------------------------------------------------------------ UTF-8 (core::str next_code_point)
__device__ __forceinline__ uint32_t utf8_next(const uint8_t *s, uint32_t n, uint32_t &i) {
  uint8_t x = s[i++];
  if (x < 128) return x;
  uint32_t init = x & 0x1F;
  uint8_t y = i < n ? s[i++] : 0;
  uint32_t ch = (init << 6) | (y & 0x3F);
  if (x >= 0xE0) {
    uint8_t z = i < n ? s[i++] : 0;
    uint32_t y_z = ((uint32_t)(y & 0x3F) << 6) | (z & 0x3F);
    ch = init << 12 | y_z;
    if (x >= 0xF0) {
      uint8_t w = i < n ? s[i++] : 0;
      ch = (init & 7) << 18 | ((y_z << 6) | (w & 0x3F));
    }
  }
  return ch;
}
__device__ __forceinline__ uint32_t ch_len16(uint32_t c) { return (c & 0xFFFF) == c ? 1 : 2; }
__device__ __forceinline__ uint32_t ch_len8(uint32_t c) {
  return c < 0x80 ? 1 : c < 0x800 ? 2 : c < 0x10000 ? 3 : 4;
}
// UTF-16 length of s[0, n) when every sequence is complete and shortest-form (then utf8_next
// consumes exactly the sequence a lead announces, ch_len8 of every char is its byte count, and
// the split at the full UTF-16 length is n): non-continuation bytes + 4-byte leads.  false =
// something else: the serial walk decides.  16-byte aligned vector loads, 64 bytes a step, the
// bytes checked four at a time in registers (SWAR: lead / continuation / overlong flags per
// byte, the expected continuations shifted in from the previous word); a 69 KB pasted string of
// the editing traces walked byte by byte over HBM took k_lp_expand 17 ms.
__device__ __forceinline__ bool str_fast16(const uint8_t *s, uint32_t n, uint32_t &len) {
  const uint64_t lo = (uint64_t)s, hi = lo + n;
  uint32_t units = 0, pl = 0, p3 = 0, p4 = 0, pe0 = 0, pf0 = 0, bad = 0; // previous word's flags
  const uint32_t H = 0x80808080u;
  for (uint64_t a = lo & ~15ull; a < hi; a += 64) {
    uint4 x[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (a + 16 * k < hi) x[k] = *(const uint4 *)(a + 16 * k);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t ws[4] = {x[k].x, x[k].y, x[k].z, x[k].w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint64_t wb = a + 16 * k + 4 * j;
        uint32_t vm = H; // valid bytes of this word (none past the end: its expectations fail there)
        if (wb < lo) vm = lo - wb >= 4 ? 0u : vm & (~0u << (8 * (uint32_t)(lo - wb)));
        if (wb >= hi) vm = 0;
        else if (wb + 4 > hi) vm &= (1u << (8 * (uint32_t)(hi - wb))) - 1u;
        const uint32_t w = ws[j];
        const uint32_t b7 = w & vm, b6 = (w << 1) & vm, b5 = (w << 2) & vm, b4 = (w << 3) & vm;
        const uint32_t cont = b7 & ~b6, lead = b7 & b6, ge3 = lead & b5, ge4 = ge3 & b4;
        const uint32_t nz1e = ((w & 0x1E1E1E1Eu) + 0x7F7F7F7Fu) & H; // bits 4..1 (5..1 of the byte) any set
        const uint32_t nz0f = ((w & 0x0F0F0F0Fu) + 0x7F7F7F7Fu) & H;
        const uint32_t nz07 = ((w & 0x07070707u) + 0x7F7F7F7Fu) & H;
        const uint32_t e0 = ge3 & ~ge4 & ~nz0f, f0 = ge4 & ~nz07;
        const uint32_t exp = (lead << 8) | (pl >> 24) | (ge3 << 16) | (p3 >> 16) | (ge4 << 24) | (p4 >> 8);
        const uint32_t e0n = (e0 << 8) | (pe0 >> 24), f0n = (f0 << 8) | (pf0 >> 24);
        bad |= (exp ^ cont) | (lead & ~b5 & ~nz1e) | (e0n & ~b5) | (f0n & ~(b5 | b4));
        units += __builtin_popcount((~b7 & vm) | lead) + __builtin_popcount(ge4);
        pl = lead;
        p3 = ge3;
        p4 = ge4;
        pe0 = e0;
        pf0 = f0;
      }
    }
  }
  bad |= (pl >> 24) | (p3 >> 16) | (p4 >> 8); // a sequence running past the end
  len = units;
  return bad == 0;
}
// SplittableString::len(Utf16) (block.rs:1391-1401)
__device__ __forceinline__ uint32_t str_len16(const uint8_t *s, uint32_t n) {
  if (n == 1) return 1;
  uint32_t k = 0, i = 0;
  if (n >= 64 && str_fast16(s, n, k)) return k;
  k = 0;
  while (i < n) k += ch_len16(utf8_next(s, n, i));
  return k;
}
// split_str(.., Utf16) -> byte offset; split_at panics off a char boundary
__device__ __forceinline__ int str_split16(const uint8_t *s, uint32_t n, uint32_t offset, uint32_t &byte_off) {
  uint32_t off = 0, u = 0, i = 0;
  while (i < n) {
    if (u >= offset) break;
    uint32_t c = utf8_next(s, n, i);
    off += ch_len8(c);
    u += ch_len16(c);
  }
  if (off > n || (off < n && (int8_t)s[off] < -0x40)) return E_PANIC;
  byte_off = off;
  return 0;
}

// ------------------------------------------------------------------ hashbrown sizing
__device__ __forceinline__ uint64_t cap_to_buckets(uint64_t cap) {
  if (cap < 8) return cap < 4 ? 4 : 8;
  uint64_t adj = cap * 8 / 7, b = 1;
  while (b < adj) b <<= 1;
  return b;
}
__device__ __forceinline__ uint64_t mask_to_cap(uint64_t mask) { return mask < 8 ? mask : ((mask + 1) / 8) * 7; }

// ------------------------------------------------------------------ f64 helpers (integer-exact)
__device__ __forceinline__ uint64_t i64_to_f64_bits(int64_t v) {
  if (v == 0) return 0;
  uint64_t sign = v < 0 ? (1ull << 63) : 0;
  uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  int lz = __clzll(m);
  int msb = 63 - lz;
  uint64_t mant;
  int e = msb;
  if (msb <= 52) {
    mant = m << (52 - msb);
  } else {
    int sh = msb - 52;
    uint64_t q = m >> sh, rem = m & ((1ull << sh) - 1), half = 1ull << (sh - 1);
    if (rem > half || (rem == half && (q & 1))) q++;
    if (q >> 53) {
      q >>= 1;
      e++;
    }
    mant = q;
  }
  return sign | ((uint64_t)(e + 1023) << 52) | (mant & ((1ull << 52) - 1));
}
// f32 -> f64 as x86 cvtss2sd (NaN quietened, payload kept)
__device__ __forceinline__ uint64_t f32_to_f64_bits(uint32_t b) {
  uint64_t sign = (uint64_t)(b >> 31) << 63;
  uint32_t ex = (b >> 23) & 0xFF, m = b & 0x7FFFFF;
  if (ex == 0xFF) return sign | (0x7FFull << 52) | ((uint64_t)m << 29) | (m ? (1ull << 51) : 0);
  if (ex == 0) {
    if (m == 0) return sign;
    int lz = __clz(m) - 9; // normalise: leading 1 to bit 23
    m <<= (lz + 1);
    int e = -126 - (lz + 1);
    return sign | ((uint64_t)(e + 1023) << 52) | ((uint64_t)(m & 0x7FFFFF) << 29);
  }
  return sign | ((uint64_t)(ex - 127 + 1023) << 52) | ((uint64_t)m << 29);
}
// Any::encode number (any.rs:136-154)
template <class W> YM_INLINE void num_encode(W &w, uint64_t bits) {
  uint64_t sign = bits >> 63;
  int ex = (int)((bits >> 52) & 0x7FF);
  uint64_t frac = bits & ((1ull << 52) - 1);
  // integral and |x| <= 2^53-1 ?
  bool integral = false;
  uint64_t ival = 0;
  if (ex == 0 && frac == 0) {
    integral = true;
    ival = 0;
  } else if (ex != 0x7FF && ex >= 1023 && ex <= 1075 - 1 + 1) {
    int e = ex - 1023; // value = (1.frac) * 2^e
    if (e <= 52) {
      uint64_t m = frac | (1ull << 52);
      uint64_t lowmask = (e == 52) ? 0 : ((1ull << (52 - e)) - 1);
      if ((m & lowmask) == 0) {
        integral = true;
        ival = m >> (52 - e);
      }
    }
  }
  if (integral && ival <= 9007199254740991ull) {
    w.u8(125);
    w_var_i64(w, sign ? -(int64_t)ival : (int64_t)ival);
    return;
  }
  // exactly representable as f32 ?
  bool f32ok = false;
  uint32_t fb = 0;
  if (ex == 0x7FF) {
    if (frac == 0) {
      f32ok = true;
      fb = (uint32_t)(sign << 31) | 0x7F800000u;
    }
  } else if (ex != 0) {
    int e = ex - 1023;
    uint64_t m = frac | (1ull << 52);
    if (e >= -126 && e <= 127) {
      if ((frac & ((1ull << 29) - 1)) == 0) {
        f32ok = true;
        fb = (uint32_t)(sign << 31) | ((uint32_t)(e + 127) << 23) | (uint32_t)(frac >> 29);
      }
    } else if (e < -126 && e >= -149) {
      int sh = -97 - e; // mf = m >> sh
      if ((m & ((1ull << sh) - 1)) == 0) {
        f32ok = true;
        fb = (uint32_t)(sign << 31) | (uint32_t)(m >> sh);
      }
    }
  }
  if (f32ok) {
    w.u8(124);
    for (int k = 3; k >= 0; k--) w.u8((uint8_t)(fb >> (8 * k)));
  } else {
    w.u8(123);
    for (int k = 7; k >= 0; k--) w.u8((uint8_t)(bits >> (8 * k)));
  }
}

// ------------------------------------------------------------------ Any (any.rs:37-83)
// Iterative walk of ONE Any value.  Validates (errors in read order), computes the
// canonical re-encoding (into W; use Counter for the size) and whether the input
// bytes already are canonical (`reenc` set when they differ).
struct AnyFrame {
  uint64_t remaining;
  uint32_t map_start; // cursor index of the first key (maps) or ~0u (arrays)
  uint32_t nkeys;
};
__device__ __noinline__ int any_skip(Cur &c); // forward
__device__ __forceinline__ bool bytes_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}
// Does a later entry of the map repeat the key [ks, ks+kn)?  c.i = start of the current
// entry's value, `rest` = entries after the current one.  Malformed tails answer false
// (the walk itself reports the error).
__device__ __noinline__ bool map_key_later(Cur c, uint64_t rest, uint32_t ks, uint32_t kn) {
  if (any_skip(c)) return false;
  for (uint64_t j = 0; j < rest; j++) {
    uint32_t l;
    bool cn;
    if (rd_var_u32(c, l, cn) || l > c.n - c.i) return false;
    if (l == kn && bytes_eq(c.p + c.i, c.p + ks, kn)) return true;
    c.i += l;
    if (any_skip(c)) return false;
  }
  return false;
}
// Output sink that can be muted: the earlier entries of a repeated Any-map key.
template <class W> struct MuteW {
  W &w;
  bool mute;
  __device__ __forceinline__ void u8(uint8_t b) {
    if (!mute) w.u8(b);
  }
  __device__ __forceinline__ void bytes(const uint8_t *s, uint32_t k) {
    if (!mute) w.bytes(s, k);
  }
};
// A map with duplicate keys holds each key once (HashMap::insert, any.rs:61-68): the entry
// count is the distinct-key count and an entry is written at its key's last occurrence.
template <bool CHECK_DUPS = true, class W> __device__ __noinline__ int any_walk(Cur &c, W &w0, bool &reenc) {
  AnyFrame st[ANY_MAX_DEPTH];
  MuteW<W> w{w0, false};
  int depth = 0, mute_at = -1; // frame depth whose current entry is muted
  for (;;) {
    // key of a map entry?
    if (depth > 0 && st[depth - 1].map_start != ~0u) {
      AnyFrame &f = st[depth - 1];
      if (mute_at == depth) { // the muted entry's value is complete
        mute_at = -1;
        w.mute = false;
      }
      if (f.remaining == 0) {
        depth--;
        if (depth == 0) return 0;
        continue;
      }
      uint32_t kl;
      bool cn;
      YM_TRY(rd_var_u32(c, kl, cn));
      if (!cn) reenc = true;
      uint32_t ks = c.i;
      YM_TRY(rd_skip(c, kl));
      f.nkeys++;
      f.remaining--;
      if (CHECK_DUPS && f.remaining && mute_at < 0 && map_key_later(c, f.remaining, ks, kl)) {
        mute_at = depth;
        w.mute = true;
      }
      w_str(w, c.p + ks, kl);
    } else if (depth > 0) {
      AnyFrame &f = st[depth - 1];
      if (f.remaining == 0) {
        depth--;
        if (depth == 0) return 0;
        continue;
      }
      f.remaining--;
    }
    // one value
    uint8_t tag;
    YM_TRY(rd_u8(c, tag));
    switch (tag) {
    case 127: case 126: case 121: case 120: w.u8(tag); break;
    case 125: {
      uint32_t s0 = c.i;
      int64_t v;
      YM_TRY(rd_var_i64(c, v));
      Counter before;
      (void)before;
      uint64_t n0 = 0;
      // canonical iff num_encode reproduces tag 125 + the same varint bytes
      struct Cmp {
        const uint8_t *p;
        uint32_t n, k;
        bool eq;
        __device__ void u8(uint8_t b) {
          if (k >= n || p[k] != b) eq = false;
          k++;
        }
        __device__ void bytes(const uint8_t *, uint32_t) {}
      } cmp{c.p + s0 - 1, c.i - s0 + 1, 0, true};
      uint64_t bits = i64_to_f64_bits(v);
      num_encode(cmp, bits);
      if (!cmp.eq || cmp.k != cmp.n) reenc = true;
      (void)n0;
      num_encode(w, bits);
      break;
    }
    case 124: {
      YM_TRY(rd_skip(c, 4));
      const uint8_t *s = c.p + c.i - 4;
      uint32_t b = (uint32_t)s[0] << 24 | (uint32_t)s[1] << 16 | (uint32_t)s[2] << 8 | s[3];
      uint64_t bits = f32_to_f64_bits(b);
      Counter cnt;
      // canonical iff it stays an f32 with identical bits
      uint32_t ex = (b >> 23) & 0xFF;
      bool nan = ex == 0xFF && (b & 0x7FFFFF);
      bool integral_safe = false;
      {
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
        integral_safe = pk.first == 125;
      }
      if (nan || integral_safe) reenc = true;
      (void)cnt;
      num_encode(w, bits);
      break;
    }
    case 123: {
      YM_TRY(rd_skip(c, 8));
      const uint8_t *s = c.p + c.i - 8;
      uint64_t bits = 0;
      for (int k = 0; k < 8; k++) bits = bits << 8 | s[k];
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
      num_encode(w, bits);
      break;
    }
    case 122: {
      YM_TRY(rd_skip(c, 8));
      w.u8(122);
      w.bytes(c.p + c.i - 8, 8);
      break;
    }
    case 119: case 116: {
      uint32_t l;
      bool cn;
      YM_TRY(rd_var_u32(c, l, cn));
      if (!cn) reenc = true;
      YM_TRY(rd_skip(c, l));
      w.u8(tag);
      w_str(w, c.p + c.i - l, l);
      break;
    }
    case 118: case 117: {
      uint64_t n;
      bool cn;
      YM_TRY(rd_var_u64(c, n, cn));
      if (!cn) reenc = true;
      if (tag == 118) {
        if (n && (n > (1ull << 40) || cap_to_buckets(n) * 49ull > ALLOC_LIMIT)) return E_PANIC;
      } else if (n > ALLOC_LIMIT / 24) {
        return E_PANIC;
      }
      w.u8(tag);
      if (depth >= ANY_MAX_DEPTH) return E_UNSUPPORTED;
      if (CHECK_DUPS && tag == 118 && n >= 2) { // distinct keys (a malformed map fails in the walk)
        Cur q = c;
        uint64_t nd = 0;
        for (uint64_t j = 0; j < n; j++) {
          uint32_t l;
          bool cn2;
          if (rd_var_u32(q, l, cn2) || l > q.n - q.i) break;
          const uint32_t ks = q.i;
          q.i += l;
          nd += !map_key_later(q, n - 1 - j, ks, l);
          if (any_skip(q)) break;
        }
        if (nd != n) reenc = true;
        w_var(w, nd < n ? nd : n);
      } else {
        w_var(w, n);
      }
      st[depth].remaining = n;
      st[depth].map_start = tag == 118 ? c.i : ~0u;
      st[depth].nkeys = 0;
      depth++;
      break;
    }
    default: return E_UNEXPECTED;
    }
    if (depth == 0) return 0;
  }
}
// skip one already-validated Any value
__device__ __noinline__ int any_skip(Cur &c) {
  uint64_t rem[ANY_MAX_DEPTH];
  uint8_t ismap[ANY_MAX_DEPTH];
  int depth = 0;
  for (;;) {
    if (depth > 0) {
      if (rem[depth - 1] == 0) {
        depth--;
        if (depth == 0) return 0;
        continue;
      }
      rem[depth - 1]--;
      if (ismap[depth - 1]) {
        uint32_t l;
        bool cn;
        YM_TRY(rd_var_u32(c, l, cn));
        YM_TRY(rd_skip(c, l));
      }
    }
    uint8_t tag;
    YM_TRY(rd_u8(c, tag));
    int64_t i64;
    uint32_t l;
    uint64_t n;
    bool cn;
    switch (tag) {
    case 127: case 126: case 121: case 120: break;
    case 125: YM_TRY(rd_var_i64(c, i64)); break;
    case 124: YM_TRY(rd_skip(c, 4)); break;
    case 123: case 122: YM_TRY(rd_skip(c, 8)); break;
    case 119: case 116:
      YM_TRY(rd_var_u32(c, l, cn));
      YM_TRY(rd_skip(c, l));
      break;
    case 118: case 117:
      YM_TRY(rd_var_u64(c, n, cn));
      if (depth >= ANY_MAX_DEPTH) return E_UNSUPPORTED;
      rem[depth] = n;
      ismap[depth] = tag == 118;
      depth++;
      break;
    default: return E_UNEXPECTED;
    }
    if (depth == 0) return 0;
  }
}

// ------------------------------------------------------------------ block parse
enum : uint8_t { BK_ITEM = 0, BK_GC = 1, BK_SKIP = 2 };
struct BlockInfo {
  uint8_t kind, ref, info;
  bool reenc;       // canonical re-encoding differs from the input bytes
  bool unsupported; // Embed / Format
  bool enc_panic;   // yrs panics when it re-encodes this block (String split off a char boundary)
  uint32_t len;     // clock length (0 => dropped Item)
  uint32_t canon;   // canonical encoded size (valid after measure)
};
// a non-ASCII String content of n bytes: its UTF-16 length and the encode_slice split at that
// length (block.rs:1718-1729): panics off a char boundary, re-encodes when shorter
__device__ __forceinline__ void str_info16(const uint8_t *s, uint32_t n, BlockInfo &bi) {
  uint32_t l16;
  if (n >= 64 && str_fast16(s, n, l16)) { // (complete shortest-form sequences: the split is s)
    bi.len = l16;
    return;
  }
  bi.len = str_len16(s, n);
  if (bi.len > 1) {
    uint32_t bo;
    if (str_split16(s, n, bi.len, bo)) bi.enc_panic = true;
    else if (bo != n) bi.reenc = true;
  }
}

struct DocOpts {
  bool skip_gc, auto_load, has_cid, enc_bytes;
  uint32_t cid_pos, cid_len;
};
// Options::decode (doc.rs:840-872): last value per key wins; map order irrelevant for the fields
YM_INLINE void doc_opts_parse(Cur a, DocOpts &o) {
  o.skip_gc = false;
  o.auto_load = false;
  o.has_cid = false;
  o.enc_bytes = true;
  if (a.i >= a.n || a.p[a.i] != 118) return;
  a.i++;
  uint64_t n;
  bool cn;
  rd_var_u64(a, n, cn);
  for (uint64_t j = 0; j < n; j++) {
    uint32_t kl;
    rd_var_u32(a, kl, cn);
    const uint8_t *k = a.p + a.i;
    a.i += kl;
    uint32_t vpos = a.i;
    const uint8_t *v = a.p + vpos;
    any_skip(a);
    auto keq = [&](const char *lit, uint32_t ln) {
      if (kl != ln) return false;
      for (uint32_t q = 0; q < ln; q++)
        if (k[q] != (uint8_t)lit[q]) return false;
      return true;
    };
    if (keq("gc", 2)) {
      if (v[0] == 120 || v[0] == 121) o.skip_gc = v[0] == 121;
    } else if (keq("autoLoad", 8)) {
      if (v[0] == 120 || v[0] == 121) o.auto_load = v[0] == 120;
    } else if (keq("collectionId", 12)) {
      if (v[0] == 119) {
        Cur s = a;
        s.i = vpos + 1;
        uint32_t l;
        rd_var_u32(s, l, cn);
        o.has_cid = true;
        o.cid_pos = s.i;
        o.cid_len = l;
      }
    } else if (keq("encoding", 8)) {
      bool one = v[0] == 122;
      for (int q = 1; q < 8 && one; q++) one = v[q] == 0;
      o.enc_bytes = one && v[8] == 1;
    }
  }
}

// Cold content kinds (JSON, Binary, Embed, Format, Type, Any, Doc, Move): out of line, cursor
// position passed and returned by value so the hot walk keeps its cursor in registers.
struct SlowRes {
  int err;
  uint32_t pos, len;
  bool reenc, unsupported;
};
// Content refs 12 / 13 exist only in the engine's internal v1x grammar (yv2.hip: lib0 v2
// Embed / Format with Any values); in lib0 v1 input they are ItemContent::decode's
// UnexpectedValue (yrs/src/block.rs:1786-1835).  Every kernel that parses content states its
// batch's grammar first with ym_set_grammar (from every lane, before any parse: no barrier
// needed).  LDS is not cleared between kernels, so a kernel that skipped the call could see a
// previous kernel's magic: every kernel including this header calls it at entry (k_decode
// and k_lean with v1: their walks bail on contents they do not restate).
static __shared__ uint32_t s_grammar_v1x;
constexpr uint32_t GRAMMAR_V1X_MAGIC = 0x76317821u;
YM_INLINE void ym_set_grammar(uint32_t v1x) { s_grammar_v1x = v1x ? GRAMMAR_V1X_MAGIC : 0u; }
YM_INLINE bool ym_grammar_v1x() { return s_grammar_v1x == GRAMMAR_V1X_MAGIC; }

__device__ __noinline__ SlowRes parse_content_slow(const uint8_t *p, uint32_t n, uint32_t pos, uint8_t ref,
                                                   bool reenc_in) {
  Cur c{p, n, pos};
  BlockInfo bi;
  bi.reenc = reenc_in;
  bi.unsupported = false;
  bi.enc_panic = false;
  bi.len = 0;
  bool cn;
  uint32_t v;
  SlowRes r{0, 0, 0, false, false};
  r.err = [&]() -> int {
  switch (ref) {
    case 1: YM_TRY(rd_var_u32(c, bi.len, cn)); bi.reenc |= !cn; return 0;
    case 2: {
      uint32_t L;
      YM_TRY(rd_var_u32(c, L, cn));
      int32_t remaining = (int32_t)L;
      if (remaining < 0) return E_NEM;
      bi.reenc = true; // re-emitted count is the element count (L + 1)
      uint32_t cnt = 0;
      while (remaining >= 0) {
        YM_TRY(rd_var_u32(c, v, cn));
        YM_TRY(rd_skip(c, v));
        cnt++;
        remaining--;
      }
      bi.len = cnt;
      return 0;
    }
    case 3: YM_TRY(rd_var_u32(c, v, cn)); bi.reenc |= !cn; YM_TRY(rd_skip(c, v)); bi.len = 1; return 0;
    case 4: {
      YM_TRY(rd_var_u32(c, v, cn));
      bi.reenc |= !cn;
      YM_TRY(rd_skip(c, v));
      const uint8_t *s = c.p + c.i - v;
      str_info16(s, v, bi);
      return 0;
    }
    case 5: case 6: { // Embed (json) / Format (key, json): re-serialised on encode
      if (ref == 6) {
        YM_TRY(rd_var_u32(c, v, cn));
        bi.reenc |= !cn;
        YM_TRY(rd_skip(c, v));
      }
      YM_TRY(rd_var_u32(c, v, cn));
      bi.reenc |= !cn;
      YM_TRY(rd_skip(c, v));
      // a text that is its own canonical form (json_plain) keeps the block's bytes: the merge
      // copies them instead of re-serialising the JSON in its sizes and write phases
      if (!json_plain(c.p + c.i - v, v)) {
        Counter cnt;
        YM_TRY(json_canon(c.p + c.i - v, v, cnt));
        bi.reenc = true;
      }
      bi.len = 1;
      return 0;
    }
    case 7: {
      uint8_t tr;
      YM_TRY(rd_u8(c, tr));
      bi.len = 1;
      switch (tr) {
      case 0: case 1: case 2: case 4: case 5: case 6: case 9: case 15: return 0;
      case 3:
        YM_TRY(rd_var_u32(c, v, cn));
        bi.reenc |= !cn;
        return rd_skip(c, v);
      case 7: {
        uint8_t f;
        uint64_t c64;
        YM_TRY(rd_u8(c, f));
        YM_TRY(rd_var_u64(c, c64, cn));
        YM_TRY(rd_var_u32(c, v, cn));
        if (f & 1) {
          YM_TRY(rd_var_u64(c, c64, cn));
          YM_TRY(rd_var_u32(c, v, cn));
        }
        bi.reenc = true;
        return 0;
      }
      default: return E_UNEXPECTED;
      }
    }
    case 8: {
      uint32_t n;
      YM_TRY(rd_var_u32(c, n, cn));
      bi.reenc |= !cn;
      if ((uint64_t)n * 24 > ALLOC_LIMIT) return E_NEM;
      Counter cnt;
      for (uint32_t k = 0; k < n; k++) YM_TRY(any_walk(c, cnt, bi.reenc));
      bi.len = n;
      return 0;
    }
    case 9: {
      YM_TRY(rd_var_u32(c, v, cn));
      YM_TRY(rd_skip(c, v));
      Counter cnt;
      bool r;
      YM_TRY(any_walk<false>(c, cnt, r));
      bi.reenc = true;
      bi.len = 1;
      return 0;
    }
    case 11: {
      int64_t f;
      uint64_t c64;
      YM_TRY(rd_var_i64(c, f));
      if (f < INT32_MIN || f > INT32_MAX) return E_VARINT;
      YM_TRY(rd_var_u64(c, c64, cn));
      YM_TRY(rd_var_u32(c, v, cn));
      if (!(f & 1)) {
        YM_TRY(rd_var_u64(c, c64, cn));
        YM_TRY(rd_var_u32(c, v, cn));
      }
      bi.reenc = true;
      bi.len = 1;
      return 0;
    }
    case 12: case 13: { // internal (yv2.hip): lib0 v2 Embed / Format, value as Any bytes
      if (!ym_grammar_v1x()) return E_UNEXPECTED;
      if (ref == 13) {
        YM_TRY(rd_var_u32(c, v, cn));
        YM_TRY(rd_skip(c, v));
      }
      Counter cnt;
      YM_TRY(any_walk(c, cnt, bi.reenc));
      bi.reenc = true;
      bi.len = 1;
      return 0;
    }
    default: return E_UNEXPECTED;
    }
  
  }();
  r.pos = c.i;
  r.len = bi.len;
  r.reenc = bi.reenc;
  r.unsupported = bi.unsupported;
  return r;
}

// Parses one block (Update::decode_block, update.rs:433-488) starting at c.i.
// defer (optional): a String content of >= defer[1] bytes is not measured here: defer[0] gets
// its byte offset in c (bi.len = its byte count as a placeholder), and the caller's workgroup
// measures it together (str16_coop); defer[0] stays ~0 otherwise.
YM_INLINE int parse_block(Cur &c, BlockInfo &bi, uint32_t *defer = nullptr) {
  uint8_t info;
  bool cn;
  YM_TRY(rd_u8(c, info));
  bi.info = info;
  bi.reenc = false;
  bi.unsupported = false;
  bi.enc_panic = false;
  if (info == 10 || info == 0) {
    bi.kind = info == 10 ? BK_SKIP : BK_GC;
    bi.ref = 0;
    YM_TRY(rd_var_u32(c, bi.len, cn));
    bi.reenc = !cn;
    return 0;
  }
  bi.kind = BK_ITEM;
  bool cant_copy = (info & 0xC0) == 0;
  uint32_t v;
  uint8_t want = info & 0xCF; // 0x10 never re-emitted; 0x20 only when parent_sub decoded
  if (info & 0x80) {
    YM_TRY(rd_var_u32(c, v, cn));
    bi.reenc |= !cn;
    YM_TRY(rd_var_u32(c, v, cn));
    bi.reenc |= !cn;
  }
  if (info & 0x40) {
    YM_TRY(rd_var_u32(c, v, cn));
    bi.reenc |= !cn;
    YM_TRY(rd_var_u32(c, v, cn));
    bi.reenc |= !cn;
  }
  if (cant_copy) {
    uint32_t pi;
    YM_TRY(rd_var_u32(c, pi, cn));
    bi.reenc |= !cn || (pi != 1 && pi != 0);
    if (pi == 1) {
      YM_TRY(rd_var_u32(c, v, cn));
      bi.reenc |= !cn;
      YM_TRY(rd_skip(c, v));
    } else {
      YM_TRY(rd_var_u32(c, v, cn));
      bi.reenc |= !cn;
      YM_TRY(rd_var_u32(c, v, cn));
      bi.reenc |= !cn;
    }
    if (info & 0x20) {
      want |= 0x20;
      YM_TRY(rd_var_u32(c, v, cn));
      bi.reenc |= !cn;
      YM_TRY(rd_skip(c, v));
    }
  }
  if (want != info) bi.reenc = true;
  uint8_t ref = info & 15;
  bi.ref = ref;
  if (ref == 1) {
    YM_TRY(rd_var_u32(c, bi.len, cn));
    bi.reenc |= !cn;
    return 0;
  }
  if (ref == 4) {
    YM_TRY(rd_var_u32(c, v, cn));
    bi.reenc |= !cn;
    YM_TRY(rd_skip(c, v));
    const uint8_t *s = c.p + c.i - v;
    if (v == 1) {
      bi.len = 1;
      return 0;
    }
    if (defer && v >= defer[1]) {
      defer[0] = c.i - v;
      bi.len = v;
      return 0;
    }
    // ASCII fast check: UTF-16 length = byte length and the full split is the whole string
    if (bytes_ascii(s, v)) {
      bi.len = v;
      return 0;
    }
    str_info16(s, v, bi);
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

// ------------------------------------------------------------------ block emit
// Canonical encoding of a (validated) block with ItemSlice offset `off`
// (slice.rs:199-251): for off > 0 the origin becomes (client, clock + off - 1).
// `len` is the decoded clock length of the original block.
template <class W>
__device__ __noinline__ int emit_block(const uint8_t *p, uint32_t n, uint32_t pos, uint64_t client, uint32_t clock,
                          uint32_t len, uint32_t off, W &w) {
  Cur c{p, n, pos};
  uint8_t info;
  bool cn;
  rd_u8(c, info);
  if (info == 10 || info == 0) {
    w.u8(info);
    w_var(w, (uint32_t)(len - off));
    return 0;
  }
  bool has_o = info & 0x80, has_r = info & 0x40, cant = (info & 0xC0) == 0;
  uint32_t oc = 0, ok = 0, rc = 0, rk = 0, pi = 0, pc = 0, pk = 0, pn_pos = 0, pn_len = 0, ps_pos = 0,
           ps_len = 0;
  bool has_ps = false;
  if (has_o) {
    rd_var_u32(c, oc, cn);
    rd_var_u32(c, ok, cn);
  }
  if (has_r) {
    rd_var_u32(c, rc, cn);
    rd_var_u32(c, rk, cn);
  }
  if (cant) {
    rd_var_u32(c, pi, cn);
    if (pi == 1) {
      rd_var_u32(c, pn_len, cn);
      pn_pos = c.i;
      c.i += pn_len;
    } else {
      rd_var_u32(c, pc, cn);
      rd_var_u32(c, pk, cn);
    }
    if (info & 0x20) {
      has_ps = true;
      rd_var_u32(c, ps_len, cn);
      ps_pos = c.i;
      c.i += ps_len;
    }
  }
  uint8_t ref = info & 15;
  uint8_t oinfo = (has_o ? 0x80 : 0) | (has_r ? 0x40 : 0) | (has_ps ? 0x20 : 0) | ref;
  uint64_t woc = oc;
  uint32_t wok = ok;
  bool worig = has_o;
  if (off != 0) {
    worig = true;
    woc = client;
    wok = clock + off - 1;
    oinfo |= 0x80;
  }
  bool wcant = (oinfo & 0xC0) == 0;
  w.u8(oinfo);
  if (worig) {
    w_var(w, woc);
    w_var(w, wok);
  }
  if (has_r) {
    w_var(w, rc);
    w_var(w, rk);
  }
  if (wcant) {
    if (pi == 1) {
      w_var(w, 1);
      w_str(w, p + pn_pos, pn_len);
    } else {
      w_var(w, 0);
      w_var(w, pc);
      w_var(w, pk);
    }
    if (has_ps) w_str(w, p + ps_pos, ps_len);
  }
  uint32_t end = len - 1;
  uint32_t v;
  switch (ref) {
  case 1: w_var(w, (uint32_t)(end - off + 1)); return 0;
  case 2: {
    uint32_t L;
    rd_var_u32(c, L, cn);
    w_var(w, (uint32_t)(end - off + 1));
    for (uint32_t k = 0; k <= L; k++) {
      rd_var_u32(c, v, cn);
      if (k >= off && k <= end) w_str(w, p + c.i, v);
      c.i += v;
    }
    return 0;
  }
  case 3:
    rd_var_u32(c, v, cn);
    w_str(w, p + c.i, v);
    return 0;
  case 4: {
    rd_var_u32(c, v, cn);
    const uint8_t *s = p + c.i;
    uint32_t sn = v, bo;
    if ((off != 0 || end != 0) && sn > 1 && bytes_ascii(s, sn)) { // UTF-16 offsets are byte offsets
      if (off > sn || end - off + 1 > sn - off) return E_PANIC; // (not reached for decoded lengths)
      s += off;
      sn = end - off + 1;
      w_str(w, s, sn);
      return 0;
    }
    if (off != 0) {
      YM_TRY(str_split16(s, sn, off, bo));
      s += bo;
      sn -= bo;
    }
    if (end != 0) {
      YM_TRY(str_split16(s, sn, (uint32_t)(end - off + 1), bo));
      sn = bo;
    }
    w_str(w, s, sn);
    return 0;
  }
  case 5: case 6: { // write_key + write_json (encoder.rs:170-179): canonical JSON text
    if (ref == 6) {
      rd_var_u32(c, v, cn);
      w_str(w, p + c.i, v);
      c.i += v;
    }
    rd_var_u32(c, v, cn);
    Counter cnt;
    YM_TRY(json_canon(p + c.i, v, cnt));
    w_var(w, cnt.n);
    return json_canon(p + c.i, v, w);
  }
  case 7: {
    uint8_t tr;
    rd_u8(c, tr);
    w.u8(tr);
    if (tr == 3) {
      rd_var_u32(c, v, cn);
      w_str(w, p + c.i, v);
    } else if (tr == 7) {
      uint8_t f;
      uint64_t sc, ec;
      uint32_t sk, ek;
      rd_u8(c, f);
      rd_var_u64(c, sc, cn);
      rd_var_u32(c, sk, cn);
      ec = sc;
      ek = sk;
      if (f & 1) {
        rd_var_u64(c, ec, cn);
        rd_var_u32(c, ek, cn);
      }
      bool single = sc == ec && sk == ek;
      w.u8((uint8_t)((single ? 0 : 1) | (f & 2) | (f & 4)));
      w_var(w, sc);
      w_var(w, sk);
      if (!single) {
        w_var(w, ec);
        w_var(w, ek);
      }
    }
    return 0;
  }
  case 12: case 13: { // internal lib0 v2 Embed / Format (yv2.hip): key, canonical Any
    if (ref == 13) {
      rd_var_u32(c, v, cn);
      w_str(w, p + c.i, v);
      c.i += v;
    }
    bool r;
    return any_walk(c, w, r);
  }
  case 8: {
    uint32_t cnt;
    rd_var_u32(c, cnt, cn);
    w_var(w, (uint32_t)(end - off + 1));
    for (uint32_t k = 0; k < cnt; k++) {
      bool r;
      if (k >= off && k <= end) {
        YM_TRY(any_walk(c, w, r));
      } else {
        any_skip(c);
      }
    }
    return 0;
  }
  case 9: {
    rd_var_u32(c, v, cn);
    uint32_t gpos = c.i, glen = v;
    c.i += v;
    DocOpts o;
    doc_opts_parse(c, o);
    w_str(w, p + gpos, glen);
    w.u8(118);
    w_var(w, o.has_cid ? 5 : 4);
    w_str(w, (const uint8_t *)"gc", 2);
    w.u8(o.skip_gc ? 121 : 120);
    if (o.has_cid) {
      w_str(w, (const uint8_t *)"collectionId", 12);
      w.u8(119);
      w_str(w, p + o.cid_pos, o.cid_len);
    }
    w_str(w, (const uint8_t *)"encoding", 8);
    w.u8(122);
    for (int k = 0; k < 7; k++) w.u8(0);
    w.u8(o.enc_bytes ? 1 : 0);
    w_str(w, (const uint8_t *)"autoLoad", 8);
    w.u8(o.auto_load ? 120 : 121);
    w_str(w, (const uint8_t *)"shouldLoad", 10);
    w.u8(o.auto_load ? 120 : 121);
    return 0;
  }
  case 11: {
    int64_t f;
    uint64_t sc, ec;
    uint32_t sk, ek;
    rd_var_i64(c, f);
    rd_var_u64(c, sc, cn);
    rd_var_u32(c, sk, cn);
    ec = sc;
    ek = sk;
    if (!(f & 1)) {
      rd_var_u64(c, ec, cn);
      rd_var_u32(c, ek, cn);
    }
    bool collapsed = sc == ec && sk == ek;
    int32_t fl = (int32_t)f;
    int32_t prio = fl >> 6;
    int32_t bb = (collapsed ? 1 : 0) | ((fl & 2) ? 2 : 0) | ((fl & 4) ? 4 : 0);
    bb |= (int32_t)((uint32_t)prio << 6);
    w_var_i64(w, bb);
    w_var(w, sc);
    w_var(w, sk);
    if (!collapsed) {
      w_var(w, ec);
      w_var(w, ek);
    }
    return 0;
  }
  }
  return E_PANIC;
}

// ------------------------------------------------------------------ small hashbrown table
// Emulates std HashMap<u64, _, BuildHasherDefault<ClientHasher>> insertion placement
// (group width 16) for tables of up to CAP buckets; slot[] holds entry index + 1.
template <int CAP> struct SmallHB {
  uint32_t buckets, items, growth_left;
  uint16_t slot[CAP];
  uint32_t keys[CAP];
  __device__ void init_empty() { buckets = items = growth_left = 0; }
  __device__ bool full(uint32_t idx) const { return slot[idx] != 0; }
  __device__ bool ctrl_empty(uint32_t idx) const {
    if (idx < buckets) return slot[idx] == 0;
    if (buckets < 16) return idx < 16 ? true : slot[idx - 16] == 0;
    return slot[idx - buckets] == 0;
  }
  __device__ uint32_t find_insert_slot(uint64_t hash) const {
    uint32_t mask = buckets - 1, pos = (uint32_t)hash & mask, stride = 0;
    for (;;) {
      for (uint32_t j = 0; j < 16; j++) {
        if (ctrl_empty(pos + j)) {
          uint32_t index = (pos + j) & mask;
          if (slot[index] != 0)
            for (uint32_t k = 0; k < buckets; k++)
              if (slot[k] == 0) return k;
          return index;
        }
      }
      stride += 16;
      pos = (pos + stride) & mask;
    }
  }
  __device__ int find(uint32_t key) const {
    for (uint32_t i = 0; i < buckets; i++)
      if (slot[i] && keys[slot[i] - 1] == key) return slot[i] - 1;
    return -1;
  }
  // returns false when the table would exceed CAP buckets
  __device__ bool resize(uint64_t cap) {
    uint64_t nb = cap_to_buckets(cap);
    if (nb > CAP) return false;
    uint16_t old[CAP];
    uint32_t ob = buckets;
    for (uint32_t i = 0; i < ob; i++) old[i] = slot[i];
    buckets = (uint32_t)nb;
    for (uint32_t i = 0; i < buckets; i++) slot[i] = 0;
    for (uint32_t i = 0; i < ob; i++)
      if (old[i]) slot[find_insert_slot(keys[old[i] - 1])] = old[i];
    growth_left = (uint32_t)mask_to_cap(buckets - 1) - items;
    return true;
  }
  __device__ bool reserve(uint64_t add) {
    if (add <= growth_left) return true;
    uint64_t full_cap = buckets ? mask_to_cap(buckets - 1) : 0;
    uint64_t need = items + add;
    return resize(need > full_cap + 1 ? need : full_cap + 1);
  }
  __device__ bool with_capacity(uint64_t n) {
    init_empty();
    if (n == 0) return true;
    uint64_t nb = cap_to_buckets(n);
    if (nb > CAP) return false;
    buckets = (uint32_t)nb;
    for (uint32_t i = 0; i < buckets; i++) slot[i] = 0;
    growth_left = (uint32_t)mask_to_cap(buckets - 1);
    return true;
  }
  __device__ void place(uint32_t key, uint32_t e) {
    keys[e] = key;
    slot[find_insert_slot(key)] = (uint16_t)(e + 1);
    items++;
    growth_left--;
  }
  // HashMap::insert: reserve(1) first, replace if present; returns entry or -1 (overflow)
  __device__ int insert(uint32_t key, uint32_t new_e, bool &existed) {
    if (!reserve(1)) return -2;
    int e = find(key);
    existed = e >= 0;
    if (existed) return e;
    place(key, new_e);
    return (int)new_e;
  }
  // HashMap::entry(..).or_insert: reserve(1) only when vacant
  __device__ int entry(uint32_t key, uint32_t new_e, bool &existed) {
    int e = find(key);
    existed = e >= 0;
    if (existed) return e;
    if (!reserve(1)) return -2;
    place(key, new_e);
    return (int)new_e;
  }
};

} // namespace ym
