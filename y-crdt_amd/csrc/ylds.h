// ylds.h — fast-shape decode of one v1 update staged in LDS.
//
// A round of NT consecutive updates of a document is one contiguous byte range in
// HBM; the workgroup copies it into LDS with coalesced dword loads, then every lane
// decodes its own update from LDS.  Varints are read branch-free: two dword reads
// (ds_read2_b32) cover the <= 5 bytes of a u32 LEB128, the terminator is found with
// a ctz over the continuation bits, so lanes stay converged whatever the varint
// lengths.  The shapes handled are the ones a text editor emits: client sections of
// GC / Skip / Deleted / ASCII String blocks (one block per update for an editor's
// transactions, many for a snapshot), any DeleteSet; anything else, and any malformed
// input, bails out (-1) and the caller runs the exact walk (ysm.h), which also owns the
// error codes.  Semantics follow Update::decode_v1
// (yrs/src/update.rs:714-749, 433-488), ItemContent::decode (yrs/src/block.rs:1786-1835)
// and IdSet::decode (yrs/src/id_set.rs:412-426), exactly as ysm.h restates them.
#pragma once
#include "ycodec.h"

namespace ym {

struct LCur {
  const uint32_t *w; // staged dwords
  uint32_t p, end;   // byte position / end (exclusive) within the staged buffer
};
YM_INLINE uint32_t lds_byte(const uint32_t *w, uint32_t p) { return (w[p >> 2] >> ((p & 3) * 8)) & 0xFF; }

// one LEB128 u32 (<= 5 bytes) with yrs' wrapping_shl semantics; false = bail
YM_INLINE bool lvar(LCur &c, uint32_t &v, bool &canon) {
  const uint32_t q = c.p >> 2, sh = (c.p & 3) * 8;
  const uint64_t d = ((uint64_t)c.w[q + 1] << 32) | c.w[q];
  const uint32_t x = (uint32_t)(d >> sh);
  const uint32_t b4 = (uint32_t)(d >> (sh + 32)) & 0xFF;
  const uint32_t stop = ~x & 0x80808080u;
  uint32_t len;
  if (stop) {
    len = (__builtin_ctz(stop) >> 3) + 1;
  } else {
    if (b4 & 0x80) return false; // longer than 5 bytes: exact walk
    len = 5;
  }
  if (c.p + len > c.end) return false;
  uint32_t val = (x & 0x7Fu) | ((x >> 1) & 0x3F80u) | ((x >> 2) & 0x1FC000u) | ((x >> 3) & 0xFE00000u);
  if (len < 4) val &= (1u << (7 * len)) - 1;
  else if (len == 5) val |= (b4 & 0x7Fu) << 28;
  const uint32_t last = len == 5 ? b4 : (x >> (8 * (len - 1))) & 0xFF;
  // minimal length <=> a one-byte varint, or a nonzero last group (that still fits in u32)
  canon = len == 1 || (last != 0 && (len != 5 || last < 16));
  v = val;
  c.p += len;
  return true;
}

// Decodes one staged update into the sink.  Returns 0, a sink error, or -1 (bail).
template <class S> YM_INLINE int fast_walk(const uint32_t *w, uint32_t start, uint32_t n, S &s) {
  LCur c{w, start, start + n};
  bool cn;
  uint32_t ncl, nds;
  if (!lvar(c, ncl, cn)) return -1;
  // every section and block takes >= 1 byte: larger counts cannot decode (the exact walk
  // reports them, including yrs' try_reserve errors for absurd counts)
  if (ncl > n) return -1;
  for (uint32_t sec = 0; sec < ncl; sec++) {
    uint32_t nb, client, clock;
    if (!lvar(c, nb, cn) || !lvar(c, client, cn) || !lvar(c, clock, cn)) return -1;
    if (nb > n) return -1;
    s.on_section(client);
    for (uint32_t j = 0; j < nb; j++) {
      const uint32_t bpos = c.p;
      if (c.p >= c.end) return -1;
      const uint32_t info = lds_byte(w, c.p++);
      BlockInfo bi;
      bi.info = (uint8_t)info;
      bi.reenc = bi.unsupported = bi.enc_panic = false;
      bi.canon = 0;
      uint32_t v;
      if (info == 10 || info == 0) {
        bi.kind = info == 10 ? BK_SKIP : BK_GC;
        bi.ref = 0;
        if (!lvar(c, bi.len, cn)) return -1;
        bi.reenc = !cn;
      } else {
        bi.kind = BK_ITEM;
        uint32_t want = info & 0xCF;
        bool ok = true;
        if (info & 0x80) {
          ok = lvar(c, v, cn) && (bi.reenc |= !cn, lvar(c, v, cn)) && (bi.reenc |= !cn, true);
        }
        if (ok && (info & 0x40)) {
          ok = lvar(c, v, cn) && (bi.reenc |= !cn, lvar(c, v, cn)) && (bi.reenc |= !cn, true);
        }
        if (!ok) return -1;
        if ((info & 0xC0) == 0) {
          uint32_t pi;
          if (!lvar(c, pi, cn)) return -1;
          bi.reenc |= !cn || (pi != 1 && pi != 0);
          if (!lvar(c, v, cn)) return -1;
          bi.reenc |= !cn;
          if (pi == 1) {
            if (v > c.end - c.p) return -1;
            c.p += v;
          } else {
            if (!lvar(c, v, cn)) return -1;
            bi.reenc |= !cn;
          }
          if (info & 0x20) {
            want |= 0x20;
            if (!lvar(c, v, cn)) return -1;
            bi.reenc |= !cn;
            if (v > c.end - c.p) return -1;
            c.p += v;
          }
        }
        if (want != info) bi.reenc = true;
        const uint32_t ref = info & 15;
        bi.ref = (uint8_t)ref;
        if (ref == 1) {
          if (!lvar(c, bi.len, cn)) return -1;
          bi.reenc |= !cn;
        } else if (ref == 4) {
          if (!lvar(c, v, cn)) return -1;
          bi.reenc |= !cn;
          if (v > c.end - c.p) return -1;
          const uint32_t s0 = c.p;
          c.p += v;
          if (v == 1) {
            bi.len = 1;
          } else {
            // any byte >= 0x80 in [s0, s0 + v)?  dword-wise: OR of the covering dwords,
            // masked to the string's bytes in the first and last dword
            uint32_t hi = 0;
            const uint32_t e0 = s0 + v, q0 = s0 >> 2, q1 = (e0 - 1) >> 2;
            for (uint32_t q = q0; q <= q1; q++) {
              uint32_t x = w[q];
              if (q == q0) x &= 0xFFFFFFFFu << (8 * (s0 & 3));
              if (q == q1 && (e0 & 3)) x &= 0xFFFFFFFFu >> (8 * (4 - (e0 & 3)));
              hi |= x;
            }
            if (hi & 0x80808080u) return -1; // UTF-16 length of non-ASCII text: exact walk
            bi.len = v;
          }
        } else {
          return -1;
        }
      }
      if (!(bi.kind == BK_ITEM && bi.len == 0)) { // Item::new -> None: dropped
        if ((uint64_t)clock + bi.len > 0xFFFFFFFFull) return -1;
        YM_TRY(s.on_block(client, clock, bi, bpos - start, c.p - bpos));
        clock += bi.len;
      }
    }
  }
  if (!lvar(c, nds, cn)) return -1;
  YM_TRY(s.on_ds_begin(nds));
  for (uint32_t i = 0; i < nds; i++) {
    uint32_t client, nr;
    if (!lvar(c, client, cn) || !lvar(c, nr, cn)) return -1;
    if (nr > n) return -1; // cannot fit: let the exact walk report it
    YM_TRY(s.on_ds_entry(client, nr));
    for (uint32_t k = 0; k < nr; k++) {
      uint32_t st, ln;
      if (!lvar(c, st, cn) || !lvar(c, ln, cn)) return -1;
      if ((uint64_t)st + ln > 0xFFFFFFFFull) return -1;
      s.on_ds_range(st, st + ln);
    }
  }
  return s.on_ds_done();
}

// Exact-walk cursor over a staged update (smwalk_update, ysm.h: same interface as WCur / LWin):
// the cold shapes fast_walk bails on (Any / Type / Binary / Embed / Format / Doc / Move content,
// non-ASCII text, multi-byte varints, malformed input) are walked where they are staged instead
// of over HBM by the merge kernels.  Varints read from one 8-byte window of the stage.
struct SCur {
  const uint8_t *p;  // the update's first byte (in the stage)
  uint32_t n, i;
  const uint32_t *w; // the stage's dwords
  uint32_t base;     // the update's byte offset in the stage
};
YM_INLINE uint32_t wc_byte(SCur &c, uint32_t pos) {
  const uint32_t o = c.base + pos;
  return (c.w[o >> 2] >> ((o & 3) * 8)) & 0xFF;
}
YM_INLINE void wc_ensure(SCur &, uint32_t) {}
YM_INLINE int wc_skip(SCur &c, uint64_t len) {
  if (len > (uint64_t)(c.n - c.i)) return E_EOS;
  c.i += (uint32_t)len;
  return 0;
}
YM_INLINE int wc_read(SCur &c, bool raw, uint32_t &v, bool &canon) {
  if (raw) {
    if (c.i >= c.n) return E_EOS;
    v = wc_byte(c, c.i++);
    return 0;
  }
  if (c.i + 8 <= c.n) {
    const uint32_t o = c.base + c.i, q = o >> 2, b = (o & 3) * 8;
    const uint64_t d0 = ((uint64_t)c.w[q + 1] << 32) | c.w[q];
    const uint64_t d = b ? (d0 >> b) | ((uint64_t)c.w[q + 2] << (64 - b)) : d0;
    const uint64_t stop = ~d & 0x8080808080808080ull;
    if (stop) {
      const uint32_t nb = ((uint32_t)__builtin_ctzll(stop) >> 3) + 1;
      uint32_t x = 0;
#pragma unroll
      for (uint32_t k = 0; k < 8; k++)
        if (k < nb) x |= ((uint32_t)(d >> (8 * k)) & 0x7Fu) << ((7 * k) & 31);
      const uint32_t last = (uint32_t)(d >> (8 * (nb - 1))) & 0xFF;
      v = x;
      canon = nb == varlen(x) && (nb != 5 || last < 16);
      c.i += nb;
      return 0;
    }
  }
  uint32_t sh = 0, nbytes = 0, b = 0;
  v = 0;
  for (;;) {
    if (c.i >= c.n) return E_EOS;
    b = wc_byte(c, c.i++);
    v |= (b & 0x7f) << (sh & 31);
    sh += 7;
    nbytes++;
    if (b < 0x80) break;
    if (sh > 70) return E_VARINT;
  }
  canon = nbytes == varlen(v) && (nbytes != 5 || b < 16);
  return 0;
}

// The lockstep form (one update per wavefront, k_decode_exact): the same cursor, with every
// position and value it returns made wave-uniform (readfirstlane).  The compiler then proves the
// walk's state uniform and compiles ysm.h's state switch to scalar branches; on the plain
// cursor the state is a VGPR, and every step ran the switch's whole exec-masked cascade
// (~1,800 cycles a step, measured with tools/walkbench.hip).
struct SCurU : SCur {};
YM_INLINE uint32_t ym_uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
YM_INLINE uint32_t wc_byte(SCurU &c, uint32_t pos) { return ym_uni(wc_byte((SCur &)c, ym_uni(pos))); }
YM_INLINE void wc_ensure(SCurU &, uint32_t) {}
YM_INLINE int wc_skip(SCurU &c, uint64_t len) {
  const int r = wc_skip((SCur &)c, len);
  c.i = ym_uni(c.i);
  return (int)ym_uni((uint32_t)r);
}
YM_INLINE int wc_read(SCurU &c, bool raw, uint32_t &v, bool &canon) {
  const int r = wc_read((SCur &)c, raw, v, canon);
  v = ym_uni(v);
  canon = ym_uni(canon ? 1u : 0u) != 0;
  c.i = ym_uni(c.i);
  return (int)ym_uni((uint32_t)r);
}

} // namespace ym
