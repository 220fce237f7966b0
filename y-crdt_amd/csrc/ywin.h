// ywin.h — register-window reader for lane-serial walks over HBM-resident updates.
//
// A lane that walks a whole (large) update byte by byte cannot afford one memory
// round trip per byte.  WCur keeps a 64-byte window of the stream in sixteen VGPRs,
// loaded with up to four 16-byte aligned vector loads issued together (a typical
// update arrives whole with its first access: a reload inside a divergent loop costs
// the wave one memory latency per iteration it happens in), and serves bytes with a
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
  uint64_t wa;      // absolute address of the window ([wa, wa + 64))
  uint32_t w0, w1, w2, w3, w4, w5, w6, w7, w8, w9, w10, w11, w12, w13, w14, w15;
};

YM_INLINE void wc_init(WCur &c, const uint8_t *p, uint32_t n) {
  c.p = p;
  c.n = n;
  c.i = 0;
  c.wa = ~0ull << 8; // forces a load on first access
  c.w0 = c.w1 = c.w2 = c.w3 = c.w4 = c.w5 = c.w6 = c.w7 = 0;
  c.w8 = c.w9 = c.w10 = c.w11 = c.w12 = c.w13 = c.w14 = c.w15 = 0;
}

YM_INLINE void wc_load(WCur &c, uint64_t a) { // a: 16-byte aligned, holds a valid byte
  const uint4 *q = (const uint4 *)a;
  uint4 x = q[0];
  c.w0 = x.x;
  c.w1 = x.y;
  c.w2 = x.z;
  c.w3 = x.w;
  const uint64_t end = (uint64_t)(c.p + c.n);
  if (a + 16 < end) {
    uint4 y = q[1];
    c.w4 = y.x;
    c.w5 = y.y;
    c.w6 = y.z;
    c.w7 = y.w;
  }
  if (a + 32 < end) {
    uint4 y = q[2];
    c.w8 = y.x;
    c.w9 = y.y;
    c.w10 = y.z;
    c.w11 = y.w;
  }
  if (a + 48 < end) {
    uint4 y = q[3];
    c.w12 = y.x;
    c.w13 = y.y;
    c.w14 = y.z;
    c.w15 = y.w;
  }
  c.wa = a;
}

// byte at stream position pos (< n).  The byte is picked out of the sixteen window
// registers with a v_perm_b32 tree: a select tree over the fields would be folded
// back into a dynamically indexed stack array (scratch) by the compiler.
YM_INLINE uint32_t wc_byte(WCur &c, uint32_t pos) {
  uint64_t a = (uint64_t)(c.p + pos);
  uint64_t off = a - c.wa;
  if (off >= 64) {
    wc_load(c, a & ~15ull);
    off = a & 15;
  }
  const uint32_t o = (uint32_t)off;
  // level 1: byte (o & 3) of dword (o >> 2 & 1) of each pair, into byte 0 (others zero)
  const uint32_t s1 = 0x0C0C0C00u | (o & 7);
  const uint32_t p0 = __builtin_amdgcn_perm(c.w1, c.w0, s1);
  const uint32_t p1 = __builtin_amdgcn_perm(c.w3, c.w2, s1);
  const uint32_t p2 = __builtin_amdgcn_perm(c.w5, c.w4, s1);
  const uint32_t p3 = __builtin_amdgcn_perm(c.w7, c.w6, s1);
  const uint32_t p4 = __builtin_amdgcn_perm(c.w9, c.w8, s1);
  const uint32_t p5 = __builtin_amdgcn_perm(c.w11, c.w10, s1);
  const uint32_t p6 = __builtin_amdgcn_perm(c.w13, c.w12, s1);
  const uint32_t p7 = __builtin_amdgcn_perm(c.w15, c.w14, s1);
  const uint32_t s2 = 0x0C0C0C00u | ((o >> 1) & 4);
  const uint32_t q0 = __builtin_amdgcn_perm(p1, p0, s2);
  const uint32_t q1 = __builtin_amdgcn_perm(p3, p2, s2);
  const uint32_t q2 = __builtin_amdgcn_perm(p5, p4, s2);
  const uint32_t q3 = __builtin_amdgcn_perm(p7, p6, s2);
  const uint32_t s3 = 0x0C0C0C00u | ((o >> 2) & 4);
  const uint32_t r0 = __builtin_amdgcn_perm(q1, q0, s3);
  const uint32_t r1 = __builtin_amdgcn_perm(q3, q2, s3);
  const uint32_t s4 = 0x0C0C0C00u | ((o >> 3) & 4);
  return __builtin_amdgcn_perm(r1, r0, s4);
}

// Make the window hold [i, i + need) (clamped to the stream end) before a burst of reads.
// Called at the top of a block / range: a wave whose lanes need reloads then waits for
// memory once per block instead of once at every byte-read site some lane misses at
// (each inlined wc_byte reload is its own divergent branch + wait).  need <= 48 is
// always satisfiable (the window starts at most 15 bytes before i).
YM_INLINE void wc_ensure(WCur &c, uint32_t need) {
  const uint64_t a = (uint64_t)(c.p + c.i), lim = (uint64_t)(c.p + c.n);
  if (a >= lim) return;
  const uint64_t want = a + need < lim ? a + need : lim;
  if (a < c.wa || want > c.wa + 64) wc_load(c, a & ~15ull);
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
  wc_ensure(c, 48);
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

} // namespace ym

namespace ym {
// walk_update (ywalk.h; Decode for Update, yrs/src/update.rs:714-749 + IdSet::decode,
// id_set.rs:412-426) on the register window; same sink interface, same error order.
struct WTrackClients {
  uint32_t c0, c1, c2, c3, n0, n1, n2, n3, n;
};
template <class S> YM_INLINE int wwalk_update(WCur &c, S &s) {
  bool cn;
  uint32_t ncl;
  YM_TRY(wc_var_u32(c, ncl, cn));
  if (ncl && cap_to_buckets(ncl) * 41ull > ALLOC_LIMIT) return E_NEM; // try_reserve, (u64, VecDeque) = 40 B
  // per-client stored-block counts for the VecDeque::try_reserve check (<= 4 distinct
  // clients tracked; more cannot reach the 2^36 B limit within a u32-sized update)
  WTrackClients tc{0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t i = 0; i < ncl; i++) {
    uint32_t nb, client, clock;
    YM_TRY(wc_var_u32(c, nb, cn));
    YM_TRY(wc_var_u32(c, client, cn));
    YM_TRY(wc_var_u32(c, clock, cn));
    uint32_t slot = 4;
    if (ncl > 1) {
      slot = tc.n > 0 && tc.c0 == client ? 0 : tc.n > 1 && tc.c1 == client ? 1 : tc.n > 2 && tc.c2 == client ? 2
             : tc.n > 3 && tc.c3 == client ? 3 : 4;
      if (slot == 4 && tc.n < 4) {
        slot = tc.n++;
        if (slot == 0) tc.c0 = client;
        else if (slot == 1) tc.c1 = client;
        else if (slot == 2) tc.c2 = client;
        else tc.c3 = client;
      }
    }
    const uint64_t existing = slot == 0 ? tc.n0 : slot == 1 ? tc.n1 : slot == 2 ? tc.n2 : slot == 3 ? tc.n3 : 0;
    if ((existing + nb) * 32ull > ALLOC_LIMIT) return E_NEM; // VecDeque<BlockCarrier>::try_reserve
    s.on_section(client);
    uint32_t stored = 0;
    for (uint32_t j = 0; j < nb; j++) {
      const uint32_t bpos = c.i;
      BlockInfo bi;
      YM_TRY(wparse_block(c, bi));
      if (bi.kind == BK_ITEM && bi.len == 0) continue; // Item::new -> None
      if ((uint64_t)clock + bi.len > 0xFFFFFFFFull) return E_PANIC;
      YM_TRY(s.on_block(client, clock, bi, bpos, c.i - bpos));
      stored++;
      clock += bi.len;
    }
    if (slot == 0) tc.n0 += stored;
    else if (slot == 1) tc.n1 += stored;
    else if (slot == 2) tc.n2 += stored;
    else if (slot == 3) tc.n3 += stored;
  }
  uint32_t nds;
  YM_TRY(wc_var_u32(c, nds, cn));
  YM_TRY(s.on_ds_begin(nds));
  for (uint32_t i = 0; i < nds; i++) {
    uint32_t client, nr;
    YM_TRY(wc_var_u32(c, client, cn));
    YM_TRY(wc_var_u32(c, nr, cn));
    YM_TRY(s.on_ds_entry(client, nr));
    for (uint32_t k = 0; k < nr; k++) {
      uint32_t st, ln;
      wc_ensure(c, 20);
      YM_TRY(wc_var_u32(c, st, cn));
      YM_TRY(wc_var_u32(c, ln, cn));
      if ((uint64_t)st + ln > 0xFFFFFFFFull) return E_PANIC;
      s.on_ds_range(st, st + ln);
    }
  }
  return s.on_ds_done();
}
} // namespace ym
