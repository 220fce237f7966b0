// yv2.hip — lib0 v2 front and back end of the MI355X engine.
//
// merge_updates_v2 / diff_updates_v2 / encode_state_vector_from_update_v2
// (yrs/src/alt.rs:35-48, 63-66, 88-97) decode with DecoderV2 and encode with EncoderV2
// around the same Update model and merge as v1.  The engine therefore runs them as:
//   k_v2_decode   one lane per update: DecoderV2 (yrs/src/updates/decoder.rs:193-504 —
//                 feature flag, 9 column buffers, IntDiffOptRle / UIntOptRle / Rle column
//                 decoders, the UTF-16 string column, the key table, diff-coded DeleteSet
//                 clocks) re-emitted as the engine's v1 grammar ("v1x"), with every check
//                 and error of Update::decode_v2 in stream order; Embed / Format values
//                 (Any bytes in v2) travel as internal content refs 12 / 13 (ycodec.h)
//   (v1 pipeline) merge / diff / state vector kernels on the v1x arena
//   k_v2_encode   one lane per document: the v1x result re-encoded with EncoderV2
//                 (yrs/src/updates/encoder.rs:182-528: column encoders, write_key with a key
//                 table that is never filled, to_vec layout), or, for state vectors, the
//                 v1 bytes behind EncoderV2's empty column header
// Device limits (status UNSUPPORTED): client ids >= 2^32 (the v1 grammar's u32 clients),
// a key-table hit beyond the first V2_KCAP keys of one update.
#include "ycodec.h"
#include "ykernels.h"
#include "ywin.h"

namespace ym {

constexpr uint32_t V2_KCAP = 64;

// ------------------------------------------------------------------ column decoders
struct ICol {
  Cur c;
  uint32_t last, count;
  int32_t diff;
};
struct UCol {
  Cur c;
  uint64_t last;
  uint32_t count;
};
struct RCol {
  Cur c;
  uint8_t last;
  int32_t count;
};
struct SCol {
  const uint8_t *s;
  uint32_t n, pos;
  UCol lens;
};

// SignedVarInt::read_signed (varint.rs): magnitude + sign (-0 is negative)
__device__ __forceinline__ int rd_var_signed(Cur &c, uint64_t &mag, bool &neg) {
  uint8_t b;
  YM_TRY(rd_u8(c, b));
  uint64_t num = b & 0x3f;
  uint32_t len = 6;
  neg = (b & 0x40) != 0;
  if (b & 0x80) {
    for (;;) {
      YM_TRY(rd_u8(c, b));
      num |= (uint64_t)(b & 0x7f) << (len & 63);
      len += 7;
      if (b < 0x80) break;
      if (len > 70) return E_VARINT;
    }
  }
  mag = num;
  return 0;
}
// IntDiffOptRleDecoder::read_u32 (decoder.rs:389-404)
__device__ __forceinline__ int icol_read(ICol &d, uint32_t &v) {
  if (d.count == 0) {
    int64_t x;
    YM_TRY(rd_var_i64(d.c, x));
    if (x < INT32_MIN || x > INT32_MAX) return E_VARINT; // read_var::<i32>
    const int32_t diff = (int32_t)x;
    d.diff = diff >> 1;
    if (diff & 1) {
      uint32_t cnt;
      bool cn;
      YM_TRY(rd_var_u32(d.c, cnt, cn));
      if (cnt > 0xFFFFFFFFu - 2) return E_PANIC; // u32 + 2 overflow
      d.count = cnt + 2;
    } else {
      d.count = 1;
    }
  }
  const int64_t nv = (int64_t)(int32_t)d.last + d.diff;
  if (nv < INT32_MIN || nv > INT32_MAX) return E_PANIC; // i32 add overflow
  d.last = (uint32_t)(int32_t)nv;
  d.count--;
  v = d.last;
  return 0;
}
// UIntOptRleDecoder::read_u64 (decoder.rs:422-437)
__device__ __forceinline__ int ucol_read(UCol &d, uint64_t &v) {
  if (d.count == 0) {
    uint64_t mag;
    bool neg;
    YM_TRY(rd_var_signed(d.c, mag, neg));
    if (neg) {
      uint32_t cnt;
      bool cn;
      YM_TRY(rd_var_u32(d.c, cnt, cn));
      if (cnt > 0xFFFFFFFFu - 2) return E_PANIC;
      d.count = cnt + 2;
    } else {
      d.count = 1;
    }
    d.last = mag;
  }
  d.count--;
  v = d.last;
  return 0;
}
// RleDecoder::read_u8 (decoder.rs:455-466)
__device__ __forceinline__ int rcol_read(RCol &d, uint8_t &v) {
  if (d.count == 0) {
    YM_TRY(rd_u8(d.c, d.last));
    if (d.c.i < d.c.n) {
      uint32_t cnt;
      bool cn;
      YM_TRY(rd_var_u32(d.c, cnt, cn));
      if ((int32_t)cnt == INT32_MAX) return E_PANIC;
      d.count = (int32_t)cnt + 1;
    } else {
      d.count = -1; // read the current value forever
    }
  }
  d.count--;
  v = d.last;
  return 0;
}
// StringDecoder::read_str (decoder.rs:489-503): `remaining` UTF-16 units over chars()
__device__ __forceinline__ int scol_read(SCol &d, uint32_t &pos, uint32_t &len) {
  uint64_t remaining;
  YM_TRY(ucol_read(d.lens, remaining));
  uint32_t i = 0, j = d.pos;
  while (j < d.n) {
    if (remaining == 0) break;
    const uint32_t ch = utf8_next(d.s, d.n, j);
    i += ch_len8(ch);
    const uint32_t u = ch_len16(ch);
    if (remaining < u) return E_PANIC; // usize underflow
    remaining -= u;
  }
  const uint32_t avail = d.n - d.pos;
  if (i > avail || (i < avail && (int8_t)d.s[d.pos + i] < -0x40)) return E_PANIC; // &start[..i]
  pos = d.pos;
  len = i;
  d.pos += i;
  return 0;
}
// DecoderV2::read_usize + read_buf (decoder.rs:246-277)
__device__ __forceinline__ int usize_buf(const uint8_t *p, uint32_t n, uint32_t &idx, uint32_t &bp, uint32_t &bl) {
  if (idx >= n) return E_VARINT;
  uint64_t num = 0;
  uint32_t len = 0;
  for (;;) {
    if (idx >= n) return E_PANIC; // buf[*idx] out of bounds
    const uint8_t b = p[idx++];
    if (len >= 64) return E_PANIC; // usize shift overflow
    num |= (uint64_t)(b & 127) << len;
    len += 7;
    if (b < 128) break;
  }
  // start + len overflows usize: panics in a debug build (add) and in a release build too
  // (the wrapped end is below start: slice index order panic)
  if (num > ~0ull - idx) return E_PANIC;
  if (num > (uint64_t)(n - idx)) return E_EOS;
  bp = idx;
  bl = (uint32_t)num;
  idx += (uint32_t)num;
  return 0;
}

struct V2Dec {
  Cur r; // rest cursor
  ICol keyc, lclk, rclk;
  UCol cli, tref, len;
  RCol info, pinfo;
  SCol str;
  uint32_t nkeys, ds_cur;
  uint32_t kpos[V2_KCAP], klen[V2_KCAP];
};
// DecoderV2::new (decoder.rs:209-244)
__device__ __forceinline__ int v2_init(V2Dec &d, const uint8_t *p, uint32_t n) {
  uint32_t idx = n > 0 ? 1 : 0; // feature flag
  uint32_t bp[9], bl[9];
  for (int k = 0; k < 9; k++) YM_TRY(usize_buf(p, n, idx, bp[k], bl[k]));
  d.r = Cur{p + idx, n - idx, 0};
  d.keyc = ICol{Cur{p + bp[0], bl[0], 0}, 0, 0, 0};
  d.cli = UCol{Cur{p + bp[1], bl[1], 0}, 0, 0};
  d.lclk = ICol{Cur{p + bp[2], bl[2], 0}, 0, 0, 0};
  d.rclk = ICol{Cur{p + bp[3], bl[3], 0}, 0, 0, 0};
  d.info = RCol{Cur{p + bp[4], bl[4], 0}, 0, 0};
  d.pinfo = RCol{Cur{p + bp[6], bl[6], 0}, 0, 0};
  d.tref = UCol{Cur{p + bp[7], bl[7], 0}, 0, 0};
  d.len = UCol{Cur{p + bp[8], bl[8], 0}, 0, 0};
  // StringDecoder::new: [usize len][string bytes][UIntOptRle lengths]
  const uint8_t *sc = p + bp[5];
  uint32_t si = 0, sp, sl;
  YM_TRY(usize_buf(sc, bl[5], si, sp, sl));
  d.str.s = sc + sp;
  d.str.n = sl;
  d.str.pos = 0;
  d.str.lens = UCol{Cur{sc, bl[5], si}, 0, 0};
  d.nkeys = 0;
  d.ds_cur = 0;
  return 0;
}
__device__ __forceinline__ int d2_len(V2Dec &d, uint32_t &v) {
  uint64_t x;
  YM_TRY(ucol_read(d.len, x));
  v = (uint32_t)x; // read_len: u64 as u32
  return 0;
}
template <class W> __device__ __forceinline__ int d2_string(V2Dec &d, W &w) {
  uint32_t pos, len;
  YM_TRY(scol_read(d.str, pos, len));
  w_var(w, len);
  w.bytes(d.str.s + pos, len);
  return 0;
}
// read_key (decoder.rs:355-364): a key clock inside the table reuses the key, else the
// next string is read and appended
template <class W> __device__ __forceinline__ int d2_key(V2Dec &d, W &w) {
  uint32_t kc;
  YM_TRY(icol_read(d.keyc, kc));
  uint32_t pos, len;
  if (kc < d.nkeys) {
    if (kc >= V2_KCAP) return E_UNSUPPORTED; // device key-table capacity
    pos = d.kpos[kc];
    len = d.klen[kc];
  } else {
    YM_TRY(scol_read(d.str, pos, len));
    if (d.nkeys < V2_KCAP) {
      d.kpos[d.nkeys] = pos;
      d.klen[d.nkeys] = len;
    }
    d.nkeys++;
  }
  w_var(w, len);
  w.bytes(d.str.s + pos, len);
  return 0;
}
// one Any value of the rest cursor, validated (Any::decode) and copied
template <class W> __device__ __forceinline__ int d2_any(V2Dec &d, W &w) {
  const uint32_t st = d.r.i;
  Counter cnt;
  bool re = false;
  YM_TRY(any_walk(d.r, cnt, re));
  w.bytes(d.r.p + st, d.r.i - st);
  return 0;
}
template <class W> __device__ __forceinline__ int d2_client(V2Dec &d, W &w) {
  uint64_t x;
  YM_TRY(ucol_read(d.cli, x));
  if (x > 0xFFFFFFFFull) return E_UNSUPPORTED; // u32 client ids in the engine's grammar
  w_var(w, x);
  return 0;
}

// Update::decode_block + ItemContent::decode over DecoderV2, emitted as v1x; `ilen` = the
// block's clock length (0 for a dropped Item)
template <class W> __device__ __forceinline__ int v2_block(V2Dec &d, W &w, uint32_t &ilen) {
  uint8_t info;
  bool cn;
  uint32_t v;
  YM_TRY(rcol_read(d.info, info));
  if (info == 10 || info == 0) {
    YM_TRY(d2_len(d, v));
    w.u8(info);
    w_var(w, v);
    ilen = v;
    return 0;
  }
  const uint8_t ref = info & 15;
  w.u8(ref == 5 ? (uint8_t)((info & 0xF0) | 12) : ref == 6 ? (uint8_t)((info & 0xF0) | 13) : info);
  if (info & 0x80) { // read_left_id
    YM_TRY(d2_client(d, w));
    YM_TRY(icol_read(d.lclk, v));
    w_var(w, v);
  }
  if (info & 0x40) { // read_right_id
    YM_TRY(d2_client(d, w));
    YM_TRY(icol_read(d.rclk, v));
    w_var(w, v);
  }
  if ((info & 0xC0) == 0) {
    uint8_t pi;
    YM_TRY(rcol_read(d.pinfo, pi));
    if (pi == 1) {
      w_var(w, 1);
      YM_TRY(d2_string(d, w));
    } else {
      w_var(w, 0);
      YM_TRY(d2_client(d, w));
      YM_TRY(icol_read(d.lclk, v));
      w_var(w, v);
    }
    if (info & 0x20) YM_TRY(d2_string(d, w));
  }
  switch (ref) {
  case 1: YM_TRY(d2_len(d, v)); w_var(w, v); ilen = v; return 0;
  case 2: {
    YM_TRY(d2_len(d, v));
    if ((int32_t)v < 0) return E_NEM;
    w_var(w, v);
    for (uint32_t k = 0; k <= v; k++) YM_TRY(d2_string(d, w));
    ilen = v + 1;
    return 0;
  }
  case 3:
    YM_TRY(rd_var_u32(d.r, v, cn));
    YM_TRY(rd_skip(d.r, v));
    w_var(w, v);
    w.bytes(d.r.p + d.r.i - v, v);
    ilen = 1;
    return 0;
  case 4: {
    uint32_t pos, len;
    YM_TRY(scol_read(d.str, pos, len));
    w_var(w, len);
    w.bytes(d.str.s + pos, len);
    ilen = str_len16(d.str.s + pos, len);
    return 0;
  }
  case 5: YM_TRY(d2_any(d, w)); ilen = 1; return 0;
  case 6: YM_TRY(d2_key(d, w)); YM_TRY(d2_any(d, w)); ilen = 1; return 0;
  case 7: {
    uint64_t t;
    YM_TRY(ucol_read(d.tref, t));
    const uint8_t tr = (uint8_t)t; // read_type_ref: u64 as u8
    w.u8(tr);
    ilen = 1;
    switch (tr) {
    case 0: case 1: case 2: case 4: case 5: case 6: case 9: case 15: return 0;
    case 3: return d2_key(d, w);
    case 7: {
      uint8_t f;
      uint64_t c64;
      YM_TRY(rd_u8(d.r, f));
      w.u8(f);
      YM_TRY(rd_var_u64(d.r, c64, cn));
      w_var(w, c64);
      YM_TRY(rd_var_u32(d.r, v, cn));
      w_var(w, v);
      if (f & 1) {
        YM_TRY(rd_var_u64(d.r, c64, cn));
        w_var(w, c64);
        YM_TRY(rd_var_u32(d.r, v, cn));
        w_var(w, v);
      }
      return 0;
    }
    default: return E_UNEXPECTED;
    }
  }
  case 8: {
    YM_TRY(d2_len(d, v));
    if ((uint64_t)v * 24 > ALLOC_LIMIT) return E_NEM;
    w_var(w, v);
    for (uint32_t k = 0; k < v; k++) YM_TRY(d2_any(d, w));
    ilen = v;
    return 0;
  }
  case 9: YM_TRY(d2_string(d, w)); YM_TRY(d2_any(d, w)); ilen = 1; return 0;
  case 11: {
    int64_t f;
    uint64_t c64;
    YM_TRY(rd_var_i64(d.r, f));
    if (f < INT32_MIN || f > INT32_MAX) return E_VARINT;
    w_var_i64(w, f);
    YM_TRY(rd_var_u64(d.r, c64, cn));
    w_var(w, c64);
    YM_TRY(rd_var_u32(d.r, v, cn));
    w_var(w, v);
    if (!(f & 1)) {
      YM_TRY(rd_var_u64(d.r, c64, cn));
      w_var(w, c64);
      YM_TRY(rd_var_u32(d.r, v, cn));
      w_var(w, v);
    }
    ilen = 1;
    return 0;
  }
  default: return E_UNEXPECTED;
  }
}

// Update::decode over DecoderV2 (update.rs:714-749, id_set.rs:412-426) -> v1x
template <class W> __device__ __forceinline__ int v2_to_v1(const uint8_t *p, uint32_t n, W &w) {
  V2Dec d;
  YM_TRY(v2_init(d, p, n));
  bool cn;
  uint32_t ncl;
  YM_TRY(rd_var_u32(d.r, ncl, cn));
  if (ncl && cap_to_buckets(ncl) * 41ull > ALLOC_LIMIT) return E_NEM; // try_reserve
  w_var(w, ncl);
  uint32_t tc[8], tn[8], ntc = 0; // blocks stored per client (VecDeque::try_reserve)
  for (uint32_t i = 0; i < ncl; i++) {
    uint32_t nb, clock;
    uint64_t client;
    YM_TRY(rd_var_u32(d.r, nb, cn));
    YM_TRY(ucol_read(d.cli, client));
    if (client > 0xFFFFFFFFull) return E_UNSUPPORTED;
    YM_TRY(rd_var_u32(d.r, clock, cn));
    uint32_t slot = 8;
    for (uint32_t q = 0; q < ntc; q++)
      if (tc[q] == (uint32_t)client) slot = q;
    if (slot == 8 && ntc < 8) {
      slot = ntc++;
      tc[slot] = (uint32_t)client;
      tn[slot] = 0;
    }
    const uint64_t existing = slot < 8 ? tn[slot] : 0;
    if ((existing + nb) * 32ull > ALLOC_LIMIT) return E_NEM;
    w_var(w, nb);
    w_var(w, client);
    w_var(w, clock);
    for (uint32_t j = 0; j < nb; j++) {
      uint32_t ilen = 0;
      YM_TRY(v2_block(d, w, ilen));
      if ((uint64_t)clock + ilen > 0xFFFFFFFFull) return E_PANIC;
      clock += ilen;
      if (slot < 8) tn[slot]++;
    }
  }
  uint32_t nds;
  YM_TRY(rd_var_u32(d.r, nds, cn));
  w_var(w, nds);
  for (uint32_t i = 0; i < nds; i++) {
    d.ds_cur = 0; // reset_ds_cur_val
    uint32_t client, nr, x;
    YM_TRY(rd_var_u32(d.r, client, cn));
    YM_TRY(rd_var_u32(d.r, nr, cn));
    w_var(w, client);
    w_var(w, nr);
    for (uint32_t k = 0; k < nr; k++) {
      YM_TRY(rd_var_u32(d.r, x, cn)); // read_ds_clock
      if ((uint64_t)d.ds_cur + x > 0xFFFFFFFFull) return E_PANIC;
      d.ds_cur += x;
      const uint32_t st = d.ds_cur;
      YM_TRY(rd_var_u32(d.r, x, cn)); // read_ds_len
      if (x == 0xFFFFFFFFu) return E_PANIC;
      const uint32_t ln = x + 1;
      if ((uint64_t)d.ds_cur + ln > 0xFFFFFFFFull) return E_PANIC;
      d.ds_cur += ln;
      w_var(w, st);
      w_var(w, ln);
    }
  }
  return 0;
}

// DecoderV2::new + StateVector::decode: position of the state vector in the rest buffer
__device__ int v2_sv_rest(const uint8_t *p, uint32_t n, uint32_t &rest) {
  V2Dec d;
  YM_TRY(v2_init(d, p, n));
  rest = (uint32_t)(d.r.p - p);
  bool cn;
  uint32_t len, clk;
  uint64_t c;
  YM_TRY(rd_var_u32(d.r, len, cn));
  if (len && (uint64_t)cap_to_buckets(len) * 17ull > ALLOC_LIMIT) return E_PANIC; // with_capacity
  for (uint32_t i = 0; i < len; i++) {
    YM_TRY(rd_var_u64(d.r, c, cn));
    YM_TRY(rd_var_u32(d.r, clk, cn));
  }
  return 0;
}

// pass 0: sizes + status per update; pass 1: v1x bytes at the scanned offsets (an empty
// update [0, 0] for a failed one, which the document's status reports)
template <bool WRITE>
__global__ void __launch_bounds__(64) k_v2_decode(const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_upd, uint64_t *sz_off,
                            uint8_t *out, uint8_t *ust) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n_upd) return;
  const uint8_t *p = bytes + upd_off[u];
  const uint32_t n = (uint32_t)(upd_off[u + 1] - upd_off[u]);
  if (!WRITE) {
    Counter cnt;
    const int e = v2_to_v1(p, n, cnt);
    ust[u] = (uint8_t)e;
    sz_off[u] = e ? 2 : cnt.n;
  } else {
    Writer w{out + sz_off[u], 0};
    if (ust[u]) {
      w.u8(0);
      w.u8(0);
    } else {
      v2_to_v1(p, n, w);
    }
  }
}
// documents: the first failing update decides (alt.rs:40-45); the merged output is dropped
__global__ void k_v2_doc_status(const uint64_t *doc_upd, const uint8_t *ust, uint32_t n_docs, uint8_t *status,
                                uint64_t *out_len) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n_docs) return;
  for (uint64_t u = doc_upd[d]; u < doc_upd[d + 1]; u++)
    if (ust[u]) {
      status[d] = ust[u];
      out_len[d] = 0;
      return;
    }
}
// diff_updates_v2 decodes the state vector first, then the update (alt.rs:88-97)
__global__ void k_v2_sv_parse(const uint8_t *sv, const uint64_t *sv_off, const uint8_t *ust, uint32_t n,
                              uint64_t *rest_off, uint64_t *rest_end, uint8_t *pre) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  uint32_t rest = 0;
  int e = 0;
  if (sv) {
    e = v2_sv_rest(sv + sv_off[d], (uint32_t)(sv_off[d + 1] - sv_off[d]), rest);
    rest_off[d] = sv_off[d] + rest;
    rest_end[d] = sv_off[d + 1];
  }
  pre[d] = (uint8_t)(e ? e : ust[d]);
}

// ------------------------------------------------------------------ EncoderV2 over a v1x document
template <class W> struct IEnc {
  uint32_t last = 0, count = 0;
  int32_t diff = 0;
  __device__ __forceinline__ void flush(W &w) {
    if (count > 0) {
      const int32_t ed = (int32_t)((uint32_t)diff << 1) | (count == 1 ? 0 : 1);
      w_var_i64(w, ed);
      if (count > 1) w_var(w, count - 2);
    }
  }
  __device__ __forceinline__ void put(W &w, uint32_t v) {
    const int32_t df = (int32_t)(v - last);
    if (diff == df) {
      last = v;
      count++;
    } else {
      flush(w);
      count = 1;
      diff = df;
      last = v;
    }
  }
};
template <class W> __device__ __forceinline__ void w_signed(W &w, uint64_t mag, bool neg) {
  w.u8((uint8_t)((mag > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (uint8_t)(mag & 63)));
  mag >>= 6;
  while (mag > 0) {
    w.u8((uint8_t)((mag > 127 ? 0x80 : 0) | (uint8_t)(mag & 127)));
    mag >>= 7;
  }
}
template <class W> struct UEnc {
  uint64_t last = 0;
  uint32_t count = 0;
  __device__ __forceinline__ void flush(W &w) {
    if (count == 1) {
      w_var_i64(w, (int64_t)last);
    } else if (count > 1) {
      w_signed(w, last, true);
      w_var(w, count - 2);
    }
  }
  __device__ __forceinline__ void put(W &w, uint64_t v) {
    if (last == v) {
      count++;
    } else {
      flush(w);
      count = 1;
      last = v;
    }
  }
};
template <class W> struct REnc {
  bool has = false;
  uint8_t last = 0;
  uint32_t count = 0;
  __device__ __forceinline__ void put(W &w, uint8_t v) {
    if (has && last == v) {
      count++;
    } else {
      if (count > 0) w_var(w, count - 1);
      count = 1;
      w.u8(v);
      last = v;
      has = true;
    }
  }
};
// UTF-16 length of a validated string: ASCII runs 16 bytes at a time (independent loads)
__device__ __forceinline__ uint32_t utf16_count(const uint8_t *s, uint32_t n) {
  if (bytes_ascii(s, n)) return n;
  uint32_t k = 0, i = 0;
  while (i < n) k += ch_len16(utf8_next(s, n, i));
  return k;
}
// the 11 streams of EncoderV2, in to_vec order of their columns (string column = sbuf + slen)
enum { S_KEY, S_CLI, S_LCLK, S_RCLK, S_INFO, S_SBUF, S_SLEN, S_PINFO, S_TREF, S_LEN, S_REST, S_N };
template <class W> struct V2Enc {
  W s[S_N];
  IEnc<W> keyc, lclk, rclk;
  UEnc<W> cli, tref, len, slen;
  REnc<W> info, pinfo;
  uint32_t seq = 0, ds_cur = 0;
  __device__ __forceinline__ void string(const uint8_t *p, uint32_t n) {
    s[S_SBUF].bytes(p, n);
    slen.put(s[S_SLEN], utf16_count(p, n));
  }
  __device__ __forceinline__ void finish() {
    keyc.flush(s[S_KEY]);
    cli.flush(s[S_CLI]);
    lclk.flush(s[S_LCLK]);
    rclk.flush(s[S_RCLK]);
    tref.flush(s[S_TREF]);
    len.flush(s[S_LEN]);
    slen.flush(s[S_SLEN]);
  }
};
// the v1x document is read through a 64-byte register window (ywin.h): a lane walking a whole
// document byte by byte over HBM waited one memory latency per byte (k_v2_encode 29.6 ms on C2)
__device__ __forceinline__ uint32_t rv(WCur &c) {
  uint32_t v = 0;
  bool cn;
  wc_var_u32(c, v, cn);
  return v;
}
__device__ __forceinline__ uint64_t rv64(WCur &c) {
  uint64_t v = 0;
  bool cn;
  wc_var_u64(c, v, cn);
  return v;
}
__device__ __forceinline__ uint8_t ru8(WCur &c) {
  uint8_t v = 0;
  wc_u8(c, v);
  return v;
}
// copies one (validated) Any value of the v1x document into the rest stream (the cold skip on
// the plain pointer)
template <class W> __device__ __forceinline__ void copy_any(WCur &c, W &rest) {
  const uint32_t st = c.i;
  Cur cc{c.p, c.n, c.i};
  any_skip(cc);
  c.i = cc.i;
  rest.bytes(c.p + st, c.i - st);
}
template <class W> __device__ __forceinline__ void e_str(V2Enc<W> &e, WCur &c) {
  const uint32_t l = rv(c);
  e.string(c.p + c.i, l);
  c.i += l;
}
// encode_diff with an empty state vector over EncoderV2 (update.rs:490-535, slice.rs:199-251,
// block.rs:1711-1754), reading the canonical v1x bytes the engine wrote
template <class W> __device__ __forceinline__ void v1x_to_v2(const uint8_t *p, uint32_t n, V2Enc<W> &e) {
  WCur c;
  wc_init(c, p, n);
  W &rest = e.s[S_REST];
  const uint32_t ncl = rv(c);
  w_var(rest, ncl);
  for (uint32_t i = 0; i < ncl; i++) {
    const uint32_t nb = rv(c);
    const uint32_t client = rv(c);
    const uint32_t clock = rv(c);
    w_var(rest, nb);
    e.cli.put(e.s[S_CLI], client);
    w_var(rest, clock);
    for (uint32_t j = 0; j < nb; j++) {
      wc_ensure(c, 32); // (the block's header in the window: one wait per block)
      const uint8_t info = ru8(c);
      if (info == 10 || info == 0) {
        e.info.put(e.s[S_INFO], info);
        e.len.put(e.s[S_LEN], rv(c));
        continue;
      }
      const uint8_t ref = info & 15;
      e.info.put(e.s[S_INFO], ref == 12 ? (uint8_t)((info & 0xF0) | 5) : ref == 13 ? (uint8_t)((info & 0xF0) | 6) : info);
      if (info & 0x80) {
        e.cli.put(e.s[S_CLI], rv(c));
        e.lclk.put(e.s[S_LCLK], rv(c));
      }
      if (info & 0x40) {
        e.cli.put(e.s[S_CLI], rv(c));
        e.rclk.put(e.s[S_RCLK], rv(c));
      }
      if ((info & 0xC0) == 0) {
        if (rv(c) == 1) {
          e.pinfo.put(e.s[S_PINFO], 1);
          e_str(e, c);
        } else {
          e.pinfo.put(e.s[S_PINFO], 0);
          e.cli.put(e.s[S_CLI], rv(c));
          e.lclk.put(e.s[S_LCLK], rv(c));
        }
        if (info & 0x20) e_str(e, c);
      }
      switch (ref) {
      case 1: e.len.put(e.s[S_LEN], rv(c)); break;
      case 2: { // written count = element count
        const uint32_t k = rv(c);
        e.len.put(e.s[S_LEN], k);
        for (uint32_t q = 0; q < k; q++) e_str(e, c);
        break;
      }
      case 3: {
        const uint32_t l = rv(c);
        w_var(rest, l);
        rest.bytes(c.p + c.i, l);
        c.i += l;
        break;
      }
      case 4: e_str(e, c); break;
      case 12: copy_any(c, rest); break;
      case 13: {
        const uint32_t l = rv(c); // write_key: key clock = sequencer (key table never filled)
        e.keyc.put(e.s[S_KEY], e.seq++);
        e.string(c.p + c.i, l);
        c.i += l;
        copy_any(c, rest);
        break;
      }
      case 7: {
        const uint8_t tr = ru8(c);
        e.tref.put(e.s[S_TREF], tr);
        if (tr == 3) {
          const uint32_t l = rv(c);
          e.keyc.put(e.s[S_KEY], e.seq++);
          e.string(c.p + c.i, l);
          c.i += l;
        } else if (tr == 7) {
          const uint8_t f = ru8(c);
          rest.u8(f);
          w_var(rest, rv64(c));
          w_var(rest, rv(c));
          if (f & 1) {
            w_var(rest, rv64(c));
            w_var(rest, rv(c));
          }
        }
        break;
      }
      case 8: {
        const uint32_t k = rv(c);
        e.len.put(e.s[S_LEN], k);
        for (uint32_t q = 0; q < k; q++) copy_any(c, rest);
        break;
      }
      case 9: e_str(e, c); copy_any(c, rest); break;
      case 11: {
        int64_t f = 0;
        Cur cc{c.p, c.n, c.i};
        rd_var_i64(cc, f);
        c.i = cc.i;
        w_var_i64(rest, f);
        w_var(rest, rv64(c));
        w_var(rest, rv(c));
        if (!(f & 1)) {
          w_var(rest, rv64(c));
          w_var(rest, rv(c));
        }
        break;
      }
      default: break;
      }
    }
  }
  // IdSet::encode over EncoderV2: per entry reset, client, count, diff-coded ranges
  const uint32_t nds = rv(c);
  w_var(rest, nds);
  for (uint32_t i = 0; i < nds; i++) {
    e.ds_cur = 0;
    w_var(rest, rv(c));
    const uint32_t nr = rv(c);
    w_var(rest, nr);
    for (uint32_t k = 0; k < nr; k++) {
      const uint32_t st = rv(c), ln = rv(c);
      w_var(rest, (uint32_t)(st - e.ds_cur)); // write_ds_clock
      e.ds_cur = st;
      w_var(rest, (uint32_t)(ln - 1)); // write_ds_len
      e.ds_cur += ln;
    }
  }
  e.finish();
}
__device__ __forceinline__ uint64_t v2_total(const V2Enc<Counter> &e) {
  uint64_t t = 1;
#pragma unroll
  for (int k = 0; k < S_N; k++) {
    if (k == S_SBUF || k == S_SLEN || k == S_REST) continue;
    t += varlen(e.s[k].n) + e.s[k].n;
  }
  const uint64_t sc = varlen(e.s[S_SBUF].n) + e.s[S_SBUF].n + e.s[S_SLEN].n;
  return t + varlen(sc) + sc + e.s[S_REST].n;
}

// mode 0: full v2 update; mode 1: state vector (EncoderV2 header of empty columns + the
// v1 state vector bytes, which the rest buffer holds unchanged)
// (64 lanes per workgroup, a document per lane: a batch of 10^4 documents is ~160 waves, so
// the encoder state may take the whole register file instead of scratch memory)
template <bool WRITE>
__global__ void __launch_bounds__(64) k_v2_encode(const uint8_t *src, const uint64_t *src_start, const uint64_t *src_len,
                            const uint8_t *status, uint32_t n_docs, uint64_t *sz_off, uint8_t *out, int mode) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n_docs) return;
  if (status[d]) {
    if (!WRITE) sz_off[d] = 0;
    return;
  }
  const uint8_t *p = src + src_start[d];
  const uint32_t n = (uint32_t)src_len[d];
  if (mode == 1) {
    if (!WRITE) {
      sz_off[d] = 11 + n;
    } else {
      uint8_t *o = out + sz_off[d];
      for (int k = 0; k < 11; k++) o[k] = k == 6 ? 1 : 0; // the string column holds "" ([1, 0])
      for (uint32_t k = 0; k < n; k++) o[11 + k] = p[k];
    }
    return;
  }
  V2Enc<Counter> ec;
  v1x_to_v2(p, n, ec);
  if (!WRITE) {
    sz_off[d] = v2_total(ec);
    return;
  }
  // column offsets from the counting walk, then the writing walk
  Writer h{out + sz_off[d], 0};
  h.u8(0); // feature flag
  V2Enc<Writer> ew;
  uint64_t at = 1;
#pragma unroll
  for (int k = 0; k < S_N; k++) {
    if (k == S_SBUF) {
      const uint64_t sc = varlen(ec.s[S_SBUF].n) + ec.s[S_SBUF].n + ec.s[S_SLEN].n;
      Writer hw{out + sz_off[d] + at, 0};
      w_var(hw, sc);
      w_var(hw, ec.s[S_SBUF].n);
      at += hw.n;
      ew.s[S_SBUF] = Writer{out + sz_off[d] + at, 0};
      at += ec.s[S_SBUF].n;
      ew.s[S_SLEN] = Writer{out + sz_off[d] + at, 0};
      at += ec.s[S_SLEN].n;
      continue;
    }
    if (k == S_SLEN) continue;
    if (k != S_REST) {
      Writer hw{out + sz_off[d] + at, 0};
      w_var(hw, ec.s[k].n);
      at += hw.n;
    }
    ew.s[k] = Writer{out + sz_off[d] + at, 0};
    at += ec.s[k].n;
  }
  v1x_to_v2(p, n, ew);
}

// ------------------------------------------------------------------ one-pass encode
// The counting walk and the writing walk above are the same lane-serial walk twice (the
// walk is the whole cost).  One pass instead: each column is written into its own scratch
// stream of V2_CAP(len) bytes (bytes past it are counted, not written), the sizes and the
// document's total come out of the same walk, and k_v2_pack lays the columns out behind the
// scanned offsets (a wave per document, coalesced copies).  A document whose column outgrew
// its stream sets `over`; the host then runs the writing walk for the batch instead.
struct V2CapW {
  uint8_t *p;
  uint64_t n, cap;
  __device__ __forceinline__ void u8(uint8_t b) {
    if (n < cap) p[n] = b;
    n++;
  }
  __device__ __forceinline__ void bytes(const uint8_t *src, uint32_t k) {
    const uint64_t lim = n >= cap ? 0 : (n + k <= cap ? k : cap - n);
    uint8_t *d = p + n;
    uint32_t i = 0;
    for (; i + 16 <= lim; i += 16) {
      uint8_t t[16];
#pragma unroll
      for (uint32_t j = 0; j < 16; j++) t[j] = src[i + j];
#pragma unroll
      for (uint32_t j = 0; j < 16; j++) d[i + j] = t[j];
    }
    for (; i < lim; i++) d[i] = src[i];
    n += k;
  }
};
__host__ __device__ inline uint64_t v2_cap(uint64_t len) { return 2 * len + 64; }
__global__ void k_v2_need(const uint64_t *src_len, const uint8_t *status, uint32_t n, uint64_t *need) {
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d < n) need[d] = status[d] ? 0 : S_N * v2_cap(src_len[d]);
}
__global__ void __launch_bounds__(64) k_v2_encode_one(const uint8_t *src, const uint64_t *src_start,
                                                      const uint64_t *src_len, const uint8_t *status, uint32_t n_docs,
                                                      const uint64_t *scr_off, uint8_t *scr, uint32_t *colsz,
                                                      uint64_t *sz, uint32_t *over) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n_docs) return;
  if (status[d]) {
    sz[d] = 0;
    return;
  }
  const uint8_t *p = src + src_start[d];
  const uint32_t n = (uint32_t)src_len[d];
  const uint64_t cap = v2_cap(n);
  uint8_t *base = scr + scr_off[d];
  V2Enc<V2CapW> e;
#pragma unroll
  for (int k = 0; k < S_N; k++) e.s[k] = V2CapW{base + (uint64_t)k * cap, 0, cap};
  v1x_to_v2(p, n, e);
  uint64_t t = 1;
  bool ov = false;
#pragma unroll
  for (int k = 0; k < S_N; k++) {
    colsz[(size_t)S_N * d + k] = (uint32_t)e.s[k].n;
    ov = ov || e.s[k].n > cap;
    if (k == S_SBUF || k == S_SLEN || k == S_REST) continue;
    t += varlen(e.s[k].n) + e.s[k].n;
  }
  const uint64_t sc = varlen(e.s[S_SBUF].n) + e.s[S_SBUF].n + e.s[S_SLEN].n;
  sz[d] = t + varlen(sc) + sc + e.s[S_REST].n;
  if (ov) atomicOr(over, 1u);
}
// the decoder in one walk too: each update's v1x bytes into a scratch slot of 4 len + 64
// bytes at 4 (upd_off[u] - upd_off[0]) + 64 u, sizes, then k_v2_xpack packs them
__global__ void __launch_bounds__(64) k_v2_decode_one(const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_upd,
                                                      uint8_t *scr, uint64_t *sz, uint8_t *ust, uint32_t *over) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n_upd) return;
  const uint8_t *p = bytes + upd_off[u];
  const uint32_t n = (uint32_t)(upd_off[u + 1] - upd_off[u]);
  V2CapW w{scr + 4 * (upd_off[u] - upd_off[0]) + 64 * u, 0, 4ull * n + 64};
  const int e = v2_to_v1(p, n, w);
  ust[u] = (uint8_t)e;
  if (e) {
    w.p[0] = 0; // an empty update [0, 0] for a failed one (the document's status reports it)
    w.p[1] = 0;
    sz[u] = 2;
  } else {
    sz[u] = w.n;
    if (w.n > w.cap) atomicOr(over, 1u);
  }
}
__global__ void __launch_bounds__(256) k_v2_xpack(const uint64_t *upd_off, uint64_t n_upd, const uint8_t *scr,
                                                  const uint64_t *off, uint8_t *out) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n_upd) return;
  Writer w{out + off[u], 0};
  w.bytes(scr + 4 * (upd_off[u] - upd_off[0]) + 64 * u, (uint32_t)(off[u + 1] - off[u]));
}
void launch_v2_decode_one(const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_upd, uint8_t *scr, uint64_t *sz,
                          uint8_t *ust, uint32_t *over, hipStream_t s) {
  if (n_upd)
    hipLaunchKernelGGL(k_v2_decode_one, dim3((unsigned)((n_upd + 63) / 64)), dim3(64), 0, s, bytes, upd_off, n_upd, scr,
                       sz, ust, over);
}
void launch_v2_xpack(const uint64_t *upd_off, uint64_t n_upd, const uint8_t *scr, const uint64_t *off, uint8_t *out,
                     hipStream_t s) {
  if (n_upd)
    hipLaunchKernelGGL(k_v2_xpack, dim3((unsigned)((n_upd + 255) / 256)), dim3(256), 0, s, upd_off, n_upd, scr, off,
                       out);
}
// lays one document's columns out in EncoderV2::to_vec order (k_v2_encode<true>'s layout)
__global__ void __launch_bounds__(64) k_v2_pack(const uint64_t *src_len, const uint8_t *status, uint32_t n_docs,
                                                const uint64_t *scr_off, const uint8_t *scr, const uint32_t *colsz,
                                                const uint64_t *out_off, uint8_t *out) {
  const uint32_t d = blockIdx.x, t = threadIdx.x;
  if (d >= n_docs || status[d]) return;
  const uint64_t cap = v2_cap(src_len[d]);
  const uint8_t *base = scr + scr_off[d];
  uint8_t *o = out + out_off[d];
  const uint32_t *cz = colsz + (size_t)S_N * d;
  uint64_t at = 1;
  if (t == 0) o[0] = 0; // feature flag
  auto copy = [&](int k) {
    const uint8_t *s = base + (uint64_t)k * cap;
    for (uint32_t q = t; q < cz[k]; q += 64) o[at + q] = s[q];
    at += cz[k];
  };
  for (int k = 0; k < S_N; k++) {
    if (k == S_SLEN) continue;
    if (k == S_SBUF) {
      const uint64_t sc = varlen(cz[S_SBUF]) + cz[S_SBUF] + cz[S_SLEN];
      Writer hw{o + at, 0};
      if (t == 0) {
        w_var(hw, sc);
        w_var(hw, (uint64_t)cz[S_SBUF]);
      }
      at += varlen(sc) + varlen(cz[S_SBUF]);
      copy(S_SBUF);
      copy(S_SLEN);
      continue;
    }
    if (k != S_REST) {
      Writer hw{o + at, 0};
      if (t == 0) w_var(hw, (uint64_t)cz[k]);
      at += varlen(cz[k]);
    }
    copy(k);
  }
}

// ------------------------------------------------------------------ launchers
void launch_v2_encode_one(const uint8_t *src, const uint64_t *src_start, const uint64_t *src_len, const uint8_t *status,
                          uint32_t n_docs, uint64_t *need, uint64_t *scr_off, uint64_t *scan_tmp, uint8_t *scr,
                          uint32_t *colsz, uint64_t *sz, uint32_t *over, hipStream_t s) {
  if (!n_docs) return;
  hipLaunchKernelGGL(k_v2_need, dim3((n_docs + 255) / 256), dim3(256), 0, s, src_len, status, n_docs, need);
  launch_scan_u64(need, scr_off, n_docs, scan_tmp, s);
  hipLaunchKernelGGL(k_v2_encode_one, dim3((n_docs + 63) / 64), dim3(64), 0, s, src, src_start, src_len, status, n_docs,
                     scr_off, scr, colsz, sz, over);
}
void launch_v2_pack(const uint64_t *src_len, const uint8_t *status, uint32_t n_docs, const uint64_t *scr_off,
                    const uint8_t *scr, const uint32_t *colsz, const uint64_t *out_off, uint8_t *out, hipStream_t s) {
  if (n_docs)
    hipLaunchKernelGGL(k_v2_pack, dim3(n_docs), dim3(64), 0, s, src_len, status, n_docs, scr_off, scr, colsz, out_off,
                       out);
}
void launch_v2_decode(bool write, const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_upd, uint64_t *sz_off,
                      uint8_t *out, uint8_t *ust, hipStream_t s) {
  if (!n_upd) return;
  const dim3 g((unsigned)((n_upd + 63) / 64)), t(64);
  if (write)
    hipLaunchKernelGGL(k_v2_decode<true>, g, t, 0, s, bytes, upd_off, n_upd, sz_off, out, ust);
  else
    hipLaunchKernelGGL(k_v2_decode<false>, g, t, 0, s, bytes, upd_off, n_upd, sz_off, out, ust);
}
void launch_v2_doc_status(const uint64_t *doc_upd, const uint8_t *ust, uint32_t n_docs, uint8_t *status,
                          uint64_t *out_len, hipStream_t s) {
  if (n_docs)
    hipLaunchKernelGGL(k_v2_doc_status, dim3((n_docs + 255) / 256), dim3(256), 0, s, doc_upd, ust, n_docs, status,
                       out_len);
}
void launch_v2_sv_parse(const uint8_t *sv, const uint64_t *sv_off, const uint8_t *ust, uint32_t n, uint64_t *rest_off,
                        uint64_t *rest_end, uint8_t *pre, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_v2_sv_parse, dim3((n + 63) / 64), dim3(64), 0, s, sv, sv_off, ust, n, rest_off, rest_end,
                       pre);
}
void launch_v2_encode(bool write, const uint8_t *src, const uint64_t *src_start, const uint64_t *src_len,
                      const uint8_t *status, uint32_t n_docs, uint64_t *sz_off, uint8_t *out, int mode, hipStream_t s) {
  if (!n_docs) return;
  const dim3 g((n_docs + 63) / 64), t(64);
  if (write)
    hipLaunchKernelGGL(k_v2_encode<true>, g, t, 0, s, src, src_start, src_len, status, n_docs, sz_off, out, mode);
  else
    hipLaunchKernelGGL(k_v2_encode<false>, g, t, 0, s, src, src_start, src_len, status, n_docs, sz_off, out, mode);
}

} // namespace ym
