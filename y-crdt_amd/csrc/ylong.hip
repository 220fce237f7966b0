// ylong.hip — stage 1 for long updates: one v1 update parsed by the whole GPU.
//
// An update is a sequence of self-delimiting blocks (Update::decode, yrs/src/update.rs:714-749;
// decode_block :433-488; ItemContent::decode yrs/src/block.rs:1786-1835): where a block ends
// depends only on where it starts.  So the parse of one long update (the reference's
// b4-update.bin: 400,972 bytes, 12,387 blocks, yrs/benches/benches.rs:456-473) is split into
//   k_lp_plan    one workgroup: the long updates k_decode listed -> chunks of LP_CH bytes
//   k_lp_chunk   workgroup per chunk: every byte position p is taken as a block start and
//                parsed speculatively (end of the block, or "not a block"); pointer doubling
//                over the chunk's positions in LDS then gives, for every p, the first block
//                boundary at or past the chunk's end reached from p, and the blocks (all /
//                stored) in between
//   k_lp_stitch  lane per update: the true chain from the first section's first block, one
//                hop per chunk (section headers and the rare content kinds the speculative
//                parse does not restate are read exactly in between) -> segments
//   k_lp_expand  workgroup per segment: the segment's block starts (hops in LDS), then every
//                block parsed exactly (parse_block) in parallel -> the OvfFill records
//   (scan)       clock lengths in block order -> every block's clock
//   k_lp_clock   lane per block: clocks into the records, u32 clock overflow check
//   k_lp_ds      workgroup per update: the DeleteSet, its range varints decoded in parallel
//                (terminator bits -> varint ordinals)
//   k_lp_final   lane per update: the record (rec_pack's shapes); anything the parallel parse
//                does not vouch for (an error anywhere, a bound exceeded) is listed for the
//                exact walker (k_decode_huge), which owns the error codes
// The records and overflow words are exactly those smwalk_update + OvfFill write (ysm.h,
// yblock.h), so every merge kernel consumes them unchanged.
#include "ycodec.h"
#include "ykernels.h"
#include "ywalk.h"
#include "yblock.h"

namespace ym {

typedef __attribute__((address_space(3))) uint32_t lp_lds_u32;

// ext[] values: end offset of the block starting at p | LP_UNST (not a stored block: Skip, or an
// Item of length 0 that Item::new drops), or LP_BAD (not a block start: a decode error from p),
// or LP_COLD (a content kind parsed only exactly: maps / nested arrays in Any, long JSON / Any
// lists, Doc, Move, weak links, the v1x internal refs)
constexpr uint32_t LP_BAD = 0xFFFFFFFFu, LP_COLD = 0xFFFFFFFEu, LP_UNST = 1u << 30, LP_OFF = LP_UNST - 1;
constexpr uint32_t LP_SPEC_LIST = 16; // JSON strings / Any values parsed speculatively

// byte reader over the chunk's LDS stage, global memory past it
struct LpRd {
  const lp_lds_u32 *w;
  uint32_t s0, se, sh; // stage holds update bytes [s0, se); s0's byte offset in the first dword
  const uint8_t *g;    // the update's first byte
  YM_INLINE uint32_t byte(uint32_t q) const {
    if (q - s0 < se - s0) {
      const uint32_t o = q - s0 + sh;
      return (w[o >> 2] >> ((o & 3) * 8)) & 0xFF;
    }
    return g[q];
  }
  // the 8 stream bytes from q (q - s0 + 8 <= se - s0): three dword reads and a funnel shift
  YM_INLINE uint64_t win8(uint32_t q) const {
    const uint32_t o = q - s0 + sh, i = o >> 2, b = (o & 3) * 8;
    const uint64_t d = ((uint64_t)w[i + 1] << 32) | w[i];
    return b ? (d >> b) | ((uint64_t)w[i + 2] << (64 - b)) : d;
  }
};

// read_var_u32 (varint.rs:244-260) at q; false = not decodable (EOS / E_VARINT).  Inside the
// stage: one 8-byte window, the terminator by ctz over the continuation bits (<= 8 bytes)
YM_INLINE bool lp_var(const LpRd &r, uint32_t &q, uint32_t L, uint32_t &v) {
  if (q - r.s0 < r.se - r.s0 && r.se - q >= 8) {
    const uint64_t d = r.win8(q);
    const uint64_t stop = ~d & 0x8080808080808080ull;
    if (stop) {
      const uint32_t n = ((uint32_t)__builtin_ctzll(stop) >> 3) + 1;
      if (n > L - q) return false;
      uint32_t x = 0;
#pragma unroll
      for (uint32_t k = 0; k < 8; k++)
        if (k < n) x |= ((uint32_t)(d >> (8 * k)) & 0x7Fu) << ((7 * k) & 31);
      v = x;
      q += n;
      return true;
    }
  }
  uint32_t x = 0, sh = 0;
  for (;;) {
    if (q >= L) return false;
    const uint32_t b = r.byte(q++);
    x |= (b & 0x7f) << (sh & 31);
    sh += 7;
    if (b < 0x80) break;
    if (sh > 70) return false;
  }
  v = x;
  return true;
}
// skip one LEB128 (read_var_i64 / u64 shape: <= 11 bytes)
YM_INLINE bool lp_skipvar(const LpRd &r, uint32_t &q, uint32_t L) {
  for (uint32_t k = 0; k < 11; k++) {
    if (q >= L) return false;
    if (r.byte(q++) < 0x80) return true;
  }
  return false;
}
YM_INLINE bool lp_skip(uint32_t &q, uint32_t L, uint32_t n) {
  if (n > L - q) return false;
  q += n;
  return true;
}

// Speculative decode_block at p (update.rs:433-488): the end of the block, or LP_BAD / LP_COLD.
// For a true block start the end equals parse_block's (k_lp_expand checks it).
YM_INLINE uint32_t lp_spec(const LpRd &r, uint32_t p, uint32_t L) {
  uint32_t q = p, v = 0;
  if (q >= L) return LP_BAD;
  const uint32_t info = r.byte(q++);
  if (info == 10 || info == 0) {
    if (!lp_var(r, q, L, v)) return LP_BAD;
    return q | (info == 10 ? LP_UNST : 0u);
  }
  if (info & 0x80)
    if (!lp_var(r, q, L, v) || !lp_var(r, q, L, v)) return LP_BAD;
  if (info & 0x40)
    if (!lp_var(r, q, L, v) || !lp_var(r, q, L, v)) return LP_BAD;
  if (!(info & 0xC0)) {
    uint32_t pi;
    if (!lp_var(r, q, L, pi)) return LP_BAD;
    if (pi == 1) {
      if (!lp_var(r, q, L, v) || !lp_skip(q, L, v)) return LP_BAD;
    } else {
      if (!lp_var(r, q, L, v) || !lp_var(r, q, L, v)) return LP_BAD;
    }
    if (info & 0x20)
      if (!lp_var(r, q, L, v) || !lp_skip(q, L, v)) return LP_BAD;
  }
  bool unst = false;
  switch (info & 15) {
  case 1: // Deleted(len)
    if (!lp_var(r, q, L, v)) return LP_BAD;
    unst = v == 0;
    break;
  case 4: // String: byte length 0 <=> UTF-16 length 0
  case 3: // Binary
  case 5: // Embed (JSON text)
    if (!lp_var(r, q, L, v) || !lp_skip(q, L, v)) return LP_BAD;
    unst = (info & 15) == 4 && v == 0;
    break;
  case 6: // Format: key, JSON text
    if (!lp_var(r, q, L, v) || !lp_skip(q, L, v)) return LP_BAD;
    if (!lp_var(r, q, L, v) || !lp_skip(q, L, v)) return LP_BAD;
    break;
  case 7: { // Type (types/mod.rs:160-200)
    if (q >= L) return LP_BAD;
    const uint32_t tr = r.byte(q++);
    if (tr == 3) {
      if (!lp_var(r, q, L, v) || !lp_skip(q, L, v)) return LP_BAD;
    } else if (tr == 7) {
      return LP_COLD; // weak link
    } else if (!(tr <= 6 || tr == 9 || tr == 15)) {
      return LP_BAD;
    }
    break;
  }
  case 2: { // JSON: L + 1 strings (block.rs:1789-1799)
    uint32_t n;
    if (!lp_var(r, q, L, n)) return LP_BAD;
    if ((int32_t)n < 0) return LP_BAD;
    if (n >= LP_SPEC_LIST) return LP_COLD;
    for (uint32_t k = 0; k <= n; k++)
      if (!lp_var(r, q, L, v) || !lp_skip(q, L, v)) return LP_BAD;
    break;
  }
  case 8: { // Any[n] (any.rs:37-83): scalars and strings only
    uint32_t n;
    if (!lp_var(r, q, L, n)) return LP_BAD;
    if (n > LP_SPEC_LIST) return LP_COLD;
    unst = n == 0;
    for (uint32_t k = 0; k < n; k++) {
      if (q >= L) return LP_BAD;
      const uint32_t tag = r.byte(q++);
      bool ok = true;
      switch (tag) {
      case 127: case 126: case 121: case 120: break;
      case 125: ok = lp_skipvar(r, q, L); break;
      case 124: ok = lp_skip(q, L, 4); break;
      case 123: case 122: ok = lp_skip(q, L, 8); break;
      case 119: case 116: ok = lp_var(r, q, L, v) && lp_skip(q, L, v); break;
      case 118: case 117: return LP_COLD;
      default: return LP_BAD;
      }
      if (!ok) return LP_BAD;
    }
    break;
  }
  case 9: case 11: case 12: case 13: return LP_COLD;
  default: return LP_BAD; // refs 0, 10, 14, 15: UnexpectedValue
  }
  return q | (unst ? LP_UNST : 0u);
}

__device__ __forceinline__ uint32_t *lp_meta(const LpArgs &a, uint32_t k) { return a.meta + (size_t)k * LP_MW; }
__device__ __forceinline__ void lp_fail(const LpArgs &a, uint32_t k) { atomicOr(&lp_meta(a, k)[LPM_FLAGS], LPF_FALLBACK); }

// ------------------------------------------------------------------ k_lp_plan
// One workgroup: the listed long updates -> chunk and position bases (scans), chunk -> update
// map; updates that do not fit the scratch (or are >= 1 GiB) go to the exact walker.
__global__ void __launch_bounds__(1024) k_lp_plan(LpArgs a) {
  __shared__ uint64_t ws[1024 / 64 + 1];
  __shared__ uint32_t s_nch, s_nt;
  const uint32_t n = a.huge[0] < HUGE_LIST ? a.huge[0] : HUGE_LIST;
  const uint64_t *list = (const uint64_t *)(a.huge + 4);
  uint64_t cbase = 0, pbase = 0, tbase = 0;
  if (threadIdx.x == 0) s_nch = s_nt = 0;
  __syncthreads();
  for (uint32_t k0 = 0; k0 < n; k0 += 1024) {
    const uint32_t k = k0 + threadIdx.x;
    uint64_t L = 0, ch = 0, nt = 0;
    if (k < n) {
      const uint64_t u = list[k];
      L = a.upd_off[u + 1] - a.upd_off[u];
      ch = (L + LP_CH - 1) / LP_CH;
      nt = (L + LP_EXT_T - 1) / LP_EXT_T;
    }
    uint64_t TL, TC, TT;
    const uint64_t preL = bscan_sum64<1024>(L < LP_UNST ? L : (uint64_t)LP_UNST, ws, TL);
    const uint64_t preC = bscan_sum64<1024>(ch, ws, TC);
    const uint64_t preT = bscan_sum64<1024>(nt, ws, TT);
    const uint64_t pb = pbase + preL, cb = cbase + preC, tb = tbase + preT;
    if (k < n) {
      uint32_t *m = lp_meta(a, k);
      const uint64_t u = list[k];
      bool fits = L < LP_UNST && pb + L <= a.pcap && cb + ch <= a.ccap && tb + nt <= a.tcap;
      m[LPM_U] = (uint32_t)u;
      m[LPM_U + 1] = (uint32_t)(u >> 32);
      m[LPM_L] = (uint32_t)L;
      m[LPM_CB] = (uint32_t)cb;
      m[LPM_NCH] = fits ? (uint32_t)ch : 0u;
      m[LPM_PB] = (uint32_t)pb;
      m[LPM_FLAGS] = fits ? 0u : LPF_FALLBACK;
      if (fits) { // (the updates that fit are a prefix of the list: the bases only grow)
        for (uint32_t c = 0; c < ch; c++) a.c2e[cb + c] = k;
        for (uint32_t q = 0; q < nt; q++) a.tmap[tb + q] = ((uint64_t)k << 32) | q;
        atomicMax(&s_nch, (uint32_t)(cb + ch));
        atomicMax(&s_nt, (uint32_t)(tb + nt));
      }
    }
    pbase += TL;
    cbase += TC;
    tbase += TT;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a.g[LPG_CHUNKS] = s_nch; // chunks of the updates that fit (every c2e entry below is written)
    a.g[LPG_TILES] = s_nt;   // k_lp_ext tiles of the updates that fit
    a.g[LPG_SEGS] = 0;
    a.g[LPG_ORDS] = 0;
    a.g[LPG_SECS] = 0;
    a.g[LPG_N] = n;
    // (huge[1], the exact walker's list count, and the 64-bit overflow bump at huge[2..3] were
    // zeroed before k_decode, whose workgroups may already have used the bump)
  }
}

// ------------------------------------------------------------------ k_lp_ext
// workgroup per LP_EXT positions of an update (the whole GPU busy even for one update; tiles
// listed per update by k_lp_plan, so a 200-byte update is one tile, not a chunk's eight): the
// bytes staged in LDS with a look-ahead, every position parsed speculatively
constexpr uint32_t LPE_NT = 256, LP_EXT = LP_EXT_T, LPE_LA = 512, LPE_PER = LP_EXT / LPE_NT;
constexpr uint32_t LPE_STAGE_W = (LP_EXT + LPE_LA) / 4 + 4;
__global__ void __launch_bounds__(LPE_NT) k_lp_ext(LpArgs a) {
  __shared__ __align__(16) uint32_t stage[LPE_STAGE_W];
  const uint32_t t = threadIdx.x, ntile = a.g[LPG_TILES];
  for (uint32_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const uint64_t tm = a.tmap[tile];
    const uint32_t *m = lp_meta(a, (uint32_t)(tm >> 32));
    const uint64_t u = m[LPM_U] | ((uint64_t)m[LPM_U + 1] << 32);
    const uint32_t L = m[LPM_L], pb = m[LPM_PB];
    const uint32_t ts = (uint32_t)tm * LP_EXT;
    __syncthreads(); // (the previous tile's stage reads)
    const uint32_t te = ts + LP_EXT < L ? ts + LP_EXT : L;
    const uint8_t *ub = a.bytes + a.upd_off[u];
    const uint64_t abs0 = (uint64_t)(ub + ts);
    const uint32_t sh = (uint32_t)(abs0 & 3);
    const uint32_t se = ts + LP_EXT + LPE_LA < L ? ts + LP_EXT + LPE_LA : L;
    const uint32_t nw = (se - ts + sh + 3) >> 2;
    const uint32_t *src = (const uint32_t *)(abs0 - sh);
    for (uint32_t q = t; q < nw; q += LPE_NT) stage[q] = src[q]; // (the arena is padded: +16 B)
    __syncthreads();
    LpRd r{(const lp_lds_u32 *)stage, ts, se, sh, ub};
#pragma unroll 1
    for (uint32_t j = 0; j < LPE_PER; j++) {
      const uint32_t p = ts + t + j * LPE_NT;
      if (p < te) a.ext[(size_t)pb + p] = lp_spec(r, p, L);
    }
  }
}

// ------------------------------------------------------------------ k_lp_chunk
// workgroup per chunk: two (jump, count) tables in LDS for the doubling
constexpr uint32_t LP_NT = 1024, LP_PER = LP_CH / LP_NT;

__global__ void __launch_bounds__(LP_NT) k_lp_chunk(LpArgs a) {
  __shared__ uint64_t jc0[LP_CH], jc1[LP_CH];
  __shared__ uint32_t s_k;
  const uint32_t t = threadIdx.x, nch = a.g[LPG_CHUNKS];
  for (uint32_t c = blockIdx.x; c < nch; c += gridDim.x) {
    __syncthreads();
    if (t == 0) s_k = a.c2e[c];
    __syncthreads();
    const uint32_t k = s_k;
    const uint32_t *m = lp_meta(a, k);
    const uint32_t L = m[LPM_L], pb = m[LPM_PB];
    const uint32_t cs = (c - m[LPM_CB]) * LP_CH, ce = cs + LP_CH < L ? cs + LP_CH : L;
    const uint32_t cn = ce - cs;
    for (uint32_t j = 0; j < LP_PER; j++) {
      const uint32_t i = t + j * LP_NT;
      if (i >= cn) break;
      const uint32_t p = cs + i;
      const uint32_t e = a.ext[(size_t)pb + p];
      uint64_t x;
      if (e >= LP_COLD) x = p; // terminal: BAD / COLD block start (self loop, no blocks)
      else x = (uint64_t)(e & LP_OFF) | ((uint64_t)(1u | ((e & LP_UNST) ? 0u : 0x10000u)) << 32);
      jc0[i] = x;
    }
    __syncthreads();
    // pointer doubling: (J, C)[p] <- (J, C)[p] + (J, C)[J] while J is inside the chunk
    uint64_t *src_t = jc0, *dst_t = jc1;
    for (uint32_t round = 0; round < 13; round++) {
      int moved = 0;
      for (uint32_t j = 0; j < LP_PER; j++) {
        const uint32_t i = t + j * LP_NT;
        if (i >= cn) break;
        uint64_t x = src_t[i];
        const uint32_t J = (uint32_t)x;
        if (J - cs < cn && J != cs + i) {
          const uint64_t y = src_t[J - cs];
          x = (y & 0xFFFFFFFFull) | ((x & ~0xFFFFFFFFull) + (y & ~0xFFFFFFFFull));
          moved |= (uint32_t)y != J;
        }
        dst_t[i] = x;
      }
      uint64_t *tmp = src_t;
      src_t = dst_t;
      dst_t = tmp;
      if (!__syncthreads_or(moved)) break;
    }
    for (uint32_t j = 0; j < LP_PER; j++) {
      const uint32_t i = t + j * LP_NT;
      if (i >= cn) break;
      a.jc[(size_t)pb + cs + i] = src_t[i];
    }
  }
}

// ------------------------------------------------------------------ k_lp_stitch
// Lane 0 of a workgroup per update: header, sections, the chain one chunk hop at a time.
__device__ __forceinline__ bool lp_seg(const LpArgs &a, uint32_t k, uint32_t start, uint32_t nb, uint32_t sec,
                                       uint32_t ord, uint32_t st) {
  const uint32_t s = atomicAdd(&a.g[LPG_SEGS], 1u);
  if (s >= a.scap) return false;
  uint32_t *w = a.seg + (size_t)s * LP_SEGW;
  w[0] = k;
  w[1] = start;
  w[2] = nb;
  w[3] = sec;
  w[4] = ord;
  w[5] = st;
  return true;
}

__global__ void __launch_bounds__(64) k_lp_stitch(LpArgs a) {
  ym_set_grammar(a.v1x);
  const uint32_t n = a.g[LPG_N];
  // a lane per update (the hops are serial within an update; medium updates are one chunk)
  for (uint32_t k = blockIdx.x * 64 + threadIdx.x; k < n; k += gridDim.x * 64) {
    uint32_t *m = lp_meta(a, k);
    if (m[LPM_FLAGS] & LPF_FALLBACK) continue;
    const uint64_t u = m[LPM_U] | ((uint64_t)m[LPM_U + 1] << 32);
    const uint32_t L = m[LPM_L], pb = m[LPM_PB];
    const uint8_t *ub = a.bytes + a.upd_off[u];
    const bool ok = [&]() -> bool {
      Cur c{ub, L, 0};
      bool cn;
      uint32_t ncl;
      if (rd_var_u32(c, ncl, cn) || ncl > L / 3) return false; // (no try_reserve failure possible)
      const uint32_t sb = atomicAdd(&a.g[LPG_SECS], ncl);
      if ((uint64_t)sb + ncl > a.seccap) return false;
      uint32_t ord = 0, st = 0, flags = ncl == 1 ? 0u : LPF_MSEC, prev = 0;
      for (uint32_t s = 0; s < ncl; s++) {
        uint32_t nb, client, clock;
        if (rd_var_u32(c, nb, cn) || rd_var_u32(c, client, cn) || rd_var_u32(c, clock, cn)) return false;
        if (s && client >= prev) flags |= LPF_ORDER; // (REC_ORDER)
        prev = client;
        if (nb > L / 2) return false;
        uint32_t *sw = a.sec + (size_t)(sb + s) * 4;
        sw[0] = client;
        sw[1] = clock;
        sw[2] = ord;
        sw[3] = k;
        uint32_t E = c.i, r = nb;
        while (r) {
          if (E >= L) return false;
          const uint32_t x = a.ext[(size_t)pb + E];
          const uint64_t y = a.jc[(size_t)pb + E]; // (issued with the ext load: one round trip a hop)
          if (x == LP_BAD) return false;
          if (x == LP_COLD) { // exact parse of this one block
            Cur cc{ub, L, E};
            BlockInfo bi;
            if (parse_block(cc, bi)) return false;
            if (!lp_seg(a, k, E, 1, sb + s, ord, st)) return false;
            ord++;
            st += !(bi.kind == BK_SKIP || (bi.kind == BK_ITEM && bi.len == 0));
            E = cc.i;
            r--;
            continue;
          }
          const uint32_t h = (uint32_t)(y >> 32) & 0xFFFF, hs = (uint32_t)(y >> 48);
          if (h <= r) {
            if (!lp_seg(a, k, E, h, sb + s, ord, st)) return false;
            ord += h;
            st += hs;
            r -= h;
            E = (uint32_t)y;
          } else { // the section ends inside this hop: r single steps
            uint32_t q = E, s2 = 0;
            for (uint32_t i = 0; i < r; i++) {
              const uint32_t xq = a.ext[(size_t)pb + q];
              s2 += !(xq & LP_UNST);
              q = xq & LP_OFF;
            }
            if (!lp_seg(a, k, E, r, sb + s, ord, st)) return false;
            ord += r;
            st += s2;
            E = q;
            r = 0;
          }
        }
        c.i = E;
      }
      m[LPM_NBALL] = ord;
      m[LPM_NB] = st;
      m[LPM_DS] = c.i;
      m[LPM_SB] = sb;
      m[LPM_NCL] = ncl;
      const uint32_t ob = atomicAdd(&a.g[LPG_ORDS], ord);
      if ((uint64_t)ob + ord > a.ocap) return false;
      m[LPM_OB] = ob;
      // overflow words: 5 per stored block, then <= 2.5 words per DeleteSet byte (entries >= 2
      // bytes: 2 words; ranges >= 2 bytes: 3 words)
      const uint64_t need = 5ull * st + 5ull * ((L - c.i) / 2 + 1) + 8;
      const uint64_t at = atomicAdd((unsigned long long *)(a.huge + 2), (unsigned long long)need);
      if (at + need > a.huge_cap) return false;
      m[LPM_OVF] = a.huge_base + (uint32_t)at;
      if (flags) atomicOr(&m[LPM_FLAGS], flags);
      return true;
    }();
    if (!ok) lp_fail(a, k);
  }
}

// str_fast16 (ycodec.h) over s[0, n) by a whole workgroup of NT lanes (a lane per aligned 16-byte chunk,
// each starting from the flags of the word before its chunk): ok = every sequence complete
// and shortest-form, units = the UTF-16 length (then str_info16 gives exactly that length, no
// re-encode, no panic); red = NT / 64 + 2 LDS words.  Uniform call, barriers inside.
template <int NT>
__device__ __forceinline__ void str16_coop(const uint8_t *s, uint32_t n, uint32_t *red, uint32_t &units, bool &ok) {
  const uint64_t lo = (uint64_t)s, hi = lo + n, a0 = lo & ~15ull;
  const uint32_t H = 0x80808080u;
  auto valid = [&](uint64_t wb) -> uint32_t {
    uint32_t vm = H;
    if (wb < lo) vm = lo - wb >= 4 ? 0u : vm & (~0u << (8 * (uint32_t)(lo - wb)));
    if (wb >= hi) vm = 0;
    else if (wb + 4 > hi) vm &= (1u << (8 * (uint32_t)(hi - wb))) - 1u;
    return vm;
  };
  uint32_t u = 0, bad = 0;
  // chunks [a0, hi + 4): the word after the last byte checks the expectations of the last one
  for (uint64_t a = a0 + 16ull * threadIdx.x; a < hi + 4; a += 16ull * NT) {
    const uint4 x = *(const uint4 *)a;
    uint32_t pl = 0, p3 = 0, p4 = 0, pe0 = 0, pf0 = 0;
    if (a > a0) { // flags of the word before the chunk
      const uint32_t w = *(const uint32_t *)(a - 4), vm = valid(a - 4);
      const uint32_t b7 = w & vm, b6 = (w << 1) & vm, b5 = (w << 2) & vm, b4 = (w << 3) & vm;
      const uint32_t nz0f = ((w & 0x0F0F0F0Fu) + 0x7F7F7F7Fu) & H, nz07 = ((w & 0x07070707u) + 0x7F7F7F7Fu) & H;
      pl = b7 & b6;
      p3 = pl & b5;
      p4 = p3 & b4;
      pe0 = p3 & ~p4 & ~nz0f;
      pf0 = p4 & ~nz07;
    }
    const uint32_t ws[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t vm = valid(a + 4 * j), w = ws[j];
      const uint32_t b7 = w & vm, b6 = (w << 1) & vm, b5 = (w << 2) & vm, b4 = (w << 3) & vm;
      const uint32_t cont = b7 & ~b6, lead = b7 & b6, ge3 = lead & b5, ge4 = ge3 & b4;
      const uint32_t nz1e = ((w & 0x1E1E1E1Eu) + 0x7F7F7F7Fu) & H;
      const uint32_t nz0f = ((w & 0x0F0F0F0Fu) + 0x7F7F7F7Fu) & H;
      const uint32_t nz07 = ((w & 0x07070707u) + 0x7F7F7F7Fu) & H;
      const uint32_t e0 = ge3 & ~ge4 & ~nz0f, f0 = ge4 & ~nz07;
      const uint32_t exp = (lead << 8) | (pl >> 24) | (ge3 << 16) | (p3 >> 16) | (ge4 << 24) | (p4 >> 8);
      const uint32_t e0n = (e0 << 8) | (pe0 >> 24), f0n = (f0 << 8) | (pf0 >> 24);
      bad |= (exp ^ cont) | (lead & ~b5 & ~nz1e) | (e0n & ~b5) | (f0n & ~(b5 | b4));
      u += __builtin_popcount((~b7 & vm) | lead) + __builtin_popcount(ge4);
      pl = lead;
      p3 = ge3;
      p4 = ge4;
      pe0 = e0;
      pf0 = f0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    u += __shfl_xor(u, o, 64);
    bad |= __shfl_xor(bad, o, 64);
  }
  const uint32_t lane = threadIdx.x & 63;
  if (threadIdx.x == 0) red[NT / 64] = red[NT / 64 + 1] = 0;
  __syncthreads();
  if (lane == 0) {
    atomicAdd(&red[NT / 64], u);
    atomicOr(&red[NT / 64 + 1], bad);
  }
  __syncthreads();
  units = red[NT / 64];
  ok = red[NT / 64 + 1] == 0;
  __syncthreads();
}

// ------------------------------------------------------------------ k_lp_expand
constexpr uint32_t LPX_NT = 256;
constexpr uint32_t LPX_LA = 1024, LPX_STAGE_W = (LP_CH + LPX_LA) / 4 + 4;
// Strings of >= LPX_COOP bytes are measured by the whole workgroup (str16_coop), up to LPX_DEF
// per tile: one lane walking the editing traces' 69 KB pasted string held k_lp_expand 3.2 ms
constexpr uint32_t LPX_COOP = 2048, LPX_DEF = 16;
__global__ void __launch_bounds__(LPX_NT) k_lp_expand(LpArgs a) {
  __shared__ uint32_t extl[LP_CH];
  __shared__ uint32_t pos[LP_CH / 2 + 1];
  __shared__ __align__(16) uint32_t stage[LPX_STAGE_W]; // the chunk's bytes (+ look-ahead)
  __shared__ uint32_t ws[LPX_NT / 64 + 2];
  __shared__ uint32_t s_flags;
  __shared__ uint32_t s_ndef, s_doff[LPX_DEF], s_dn[LPX_DEF], s_dlen[LPX_DEF];
  ym_set_grammar(a.v1x);
  const uint32_t t = threadIdx.x, nseg = a.g[LPG_SEGS] < a.scap ? a.g[LPG_SEGS] : a.scap;
  for (uint32_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const uint32_t *sw = a.seg + (size_t)s * LP_SEGW;
    const uint32_t k = sw[0], E = sw[1], nb = sw[2], sec = sw[3], ord0 = sw[4], st0 = sw[5];
    uint32_t *m = lp_meta(a, k);
    // (other segments of the update may set the flag meanwhile: one read, broadcast, so the
    // workgroup's barriers stay uniform)
    __syncthreads();
    if (t == 0) s_flags = m[LPM_FLAGS];
    __syncthreads();
    if (s_flags & LPF_FALLBACK) continue;
    const uint64_t u = m[LPM_U] | ((uint64_t)m[LPM_U + 1] << 32);
    const uint32_t L = m[LPM_L], pb = m[LPM_PB], ovb = m[LPM_OVF], ob = m[LPM_OB], nbs = m[LPM_NB];
    const uint32_t client = a.sec[(size_t)sec * 4];
    const uint8_t *ub = a.bytes + a.upd_off[u];
    const uint32_t cs = E - E % LP_CH, cn = (cs + LP_CH < L ? cs + LP_CH : L) - cs;
    __syncthreads();
    for (uint32_t i = t; i < cn; i += LPX_NT) extl[i] = a.ext[(size_t)pb + cs + i];
    // the chunk's bytes: blocks that end inside the stage are parsed from LDS (the exact parse
    // reads byte by byte: dependent global loads otherwise)
    const uint64_t abs0 = (uint64_t)(ub + cs);
    const uint32_t sh = (uint32_t)(abs0 & 3);
    const uint32_t se = cs + LP_CH + LPX_LA < L ? cs + LP_CH + LPX_LA : L;
    {
      const uint32_t nw = (se - cs + sh + 3) >> 2;
      const uint32_t *src = (const uint32_t *)(abs0 - sh);
      for (uint32_t q = t; q < nw; q += LPX_NT) stage[q] = src[q];
    }
    // lb[q - cs] = update byte q for q in [cs, se); positions are passed relative to cs (a
    // pointer below the LDS array would leave the LDS aperture once cast to a flat address)
    const uint8_t *lb = (const uint8_t *)stage + sh;
    if (t == 0) s_flags = 0;
    __syncthreads();
    if (t == 0) { // the segment's block starts: hops inside the chunk (nb <= CH / 2)
      uint32_t q = E;
      for (uint32_t i = 0; i < nb; i++) {
        pos[i] = q;
        if (i + 1 < nb) q = extl[q - cs] & LP_OFF;
      }
    }
    __syncthreads();
    uint32_t flags = 0, stc = st0;
    for (uint32_t i0 = 0; i0 < nb; i0 += LPX_NT) {
      const uint32_t i = i0 + t;
      bool stored = false;
      BlockInfo bi;
      bi.len = 0;
      uint32_t p = 0, end = 0;
      if (t == 0) s_ndef = 0;
      __syncthreads();
      uint32_t dfr[2] = {~0u, LPX_COOP}, dq = LPX_DEF;
      int perr = 0;
      if (i < nb) {
        p = pos[i];
        const uint32_t x0 = extl[p - cs];
        const bool in_lds = x0 < LP_COLD && (x0 & LP_OFF) <= se;
        Cur cc = in_lds ? Cur{lb, L - cs, p - cs} : Cur{ub, L, p};
        perr = parse_block(cc, bi, dfr);
        end = cc.i + (in_lds ? cs : 0u);
        if (!perr && dfr[0] != ~0u) { // a long String: measured below by the workgroup
          dfr[0] += in_lds ? cs : 0u;
          dq = atomicAdd(&s_ndef, 1u);
          if (dq < LPX_DEF) {
            s_doff[dq] = dfr[0];
            s_dn[dq] = dfr[1] = bi.len;
          }
        }
      }
      __syncthreads();
      {
        const uint32_t nd = s_ndef < LPX_DEF ? s_ndef : LPX_DEF;
        for (uint32_t q = 0; q < nd; q++) {
          uint32_t units;
          bool ok;
          str16_coop<LPX_NT>(ub + s_doff[q], s_dn[q], ws, units, ok);
          if (t == 0) s_dlen[q] = ok ? units : ~0u;
        }
        __syncthreads();
      }
      if (i < nb) {
        if (!perr && dfr[0] != ~0u) {
          const uint32_t r = dq < LPX_DEF ? s_dlen[dq] : ~0u;
          if (r != ~0u) bi.len = r;
          else str_info16(ub + dfr[0], bi.len, bi); // not complete shortest-form (or a 17th): the serial walk
        }
        if (perr) {
          flags |= LPF_FALLBACK;
        } else {
          stored = !(bi.kind == BK_SKIP || (bi.kind == BK_ITEM && bi.len == 0));
          const uint32_t x = extl[p - cs];
          if (x != LP_COLD && (x == LP_BAD || (x & LP_OFF) != end || !(x & LP_UNST) != stored))
            flags |= LPF_FALLBACK; // (the speculative and exact parses disagree: cannot happen)
          if (bi.unsupported) flags |= LPF_UNSUP;
          if (bi.kind == BK_SKIP) flags |= LPF_SKIP;
          if (bi.kind == BK_GC && bi.len == 0) flags |= LPF_ZGC;
          if (bi.enc_panic) flags |= LPF_PANIC;
          if (bi.kind == BK_ITEM && bi.ref != 1 && bi.ref != 4) flags |= LPF_RICH;
        }
        a.blen[(size_t)ob + ord0 + i] = bi.len;
      }
      uint32_t tot;
      const uint32_t pre = bscan_sum<LPX_NT>(stored ? 1u : 0u, ws, tot);
      if (i < nb) {
        const size_t og = (size_t)ob + ord0 + i;
        if (stored && stc + pre < nbs) { // (bound: cannot fail when the two parses agree)
          const uint32_t at = ovb + 5 * (stc + pre);
          uint32_t *w = a.ovf + at;
          w[0] = client;
          w[1] = 0; // clock: k_lp_clock
          w[2] = bi.len;
          w[3] = p;
          w[4] = (uint32_t)bi.kind | (bi.reenc ? 4u : 0u) | (bi.enc_panic ? 8u : 0u) | ((end - p) << 8);
          a.omap[og] = at + 1;
        } else {
          a.omap[og] = 0;
        }
      }
      stc += tot;
    }
    // flags of the workgroup -> one atomic
    for (int o = 32; o > 0; o >>= 1) flags |= __shfl_xor(flags, o, 64);
    if ((t & 63) == 0 && flags) atomicOr(&s_flags, flags);
    __syncthreads();
    if (t == 0 && s_flags) atomicOr(&m[LPM_FLAGS], s_flags);
  }
}

// ------------------------------------------------------------------ k_lp_clock
// workgroup per segment, lane per block: clock = section clock + the clock lengths of the
// section's earlier blocks (scan over block ordinals); u32 overflow (update.rs:740) -> exact walker
__global__ void __launch_bounds__(256) k_lp_clock(LpArgs a) {
  const uint32_t nseg = a.g[LPG_SEGS] < a.scap ? a.g[LPG_SEGS] : a.scap;
  for (uint32_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const uint32_t *sw = a.seg + (size_t)s * LP_SEGW;
    const uint32_t k = sw[0], nb = sw[2], sec = sw[3], ord0 = sw[4];
    uint32_t *m = lp_meta(a, k);
    if (m[LPM_FLAGS] & LPF_FALLBACK) continue; // (final: k_lp_expand has finished)
    const uint32_t *sc = a.sec + (size_t)sec * 4;
    const uint64_t ob = m[LPM_OB], first = ob + sc[2], c0 = sc[1];
    for (uint32_t i = threadIdx.x; i < nb; i += 256) {
      const uint64_t o = ob + ord0 + i;
      const uint64_t clock = c0 + (a.sblen[o] - a.sblen[first]);
      if (clock + a.blen[o] > 0xFFFFFFFFull) {
        lp_fail(a, k);
        continue;
      }
      const uint32_t at = a.omap[o];
      if (at) a.ovf[at] = (uint32_t)clock; // word 1 of the record at at - 1
    }
  }
}

// ------------------------------------------------------------------ k_lp_ds
// Workgroup per update: IdSet::decode (id_set.rs:412-426) from the DeleteSet offset.  Entry
// headers are read by one lane; an entry's 2 * nr range varints are decoded in tiles of
// LPD_NT * 16 bytes: a byte ends a varint iff < 0x80, the varint ordinal of a byte is the count
// of terminators before it.
constexpr uint32_t LPD_NT = 1024, LPD_B = 16;
__device__ __forceinline__ bool lp_dvar(const uint8_t *p, uint32_t L, uint32_t q, uint32_t &v) {
  uint32_t x = 0, sh = 0;
  for (;;) {
    if (q >= L) return false;
    const uint32_t b = p[q++];
    x |= (b & 0x7f) << (sh & 31);
    sh += 7;
    if (b < 0x80) break;
    if (sh > 70) return false;
  }
  v = x;
  return true;
}

__global__ void __launch_bounds__(LPD_NT) k_lp_ds(LpArgs a) {
  __shared__ uint32_t ws[LPD_NT / 64 + 1];
  __shared__ uint32_t s_hdr[4]; // ok, nr, pos
  __shared__ uint32_t s_fail, s_cl[DS_SMALL], s_code[DS_SMALL];
  __shared__ uint32_t tileb[LPD_NT * LPD_B / 4 + 4];
  const uint32_t t = threadIdx.x, n = a.g[LPG_N];
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    uint32_t *m = lp_meta(a, k);
    __syncthreads();
    if (m[LPM_FLAGS] & LPF_FALLBACK) continue; // (uniform: no kernel writes the flag meanwhile)
    const uint64_t u = m[LPM_U] | ((uint64_t)m[LPM_U + 1] << 32);
    const uint32_t L = m[LPM_L], NB = m[LPM_NB];
    const uint8_t *ub = a.bytes + a.upd_off[u];
    uint32_t *ov = a.ovf + m[LPM_OVF] + 5 * NB;
    if (t == 0) {
      Cur c{ub, L, m[LPM_DS]};
      bool cn;
      uint32_t nds;
      s_fail = rd_var_u32(c, nds, cn) || nds > L / 2;
      s_hdr[0] = nds;
      s_hdr[2] = c.i;
    }
    __syncthreads();
    if (s_fail) {
      if (t == 0) lp_fail(a, k);
      continue;
    }
    const uint32_t nds = s_hdr[0];
    const bool big = nds > DS_SMALL;
    uint32_t *rw = ov + 2 * nds; // range words
    uint32_t rtot = 0;
    for (uint32_t e = 0; e < nds; e++) {
      if (t == 0) {
        Cur c{ub, L, s_hdr[2]};
        bool cn;
        uint32_t client, nr;
        if (rd_var_u32(c, client, cn) || rd_var_u32(c, nr, cn) || nr > L / 2) {
          s_fail = 1;
        } else {
          if (!big) ov[e] = client;
          if (e < DS_SMALL) s_cl[e] = client;
          s_hdr[1] = nr;
          s_hdr[2] = c.i;
        }
      }
      __syncthreads();
      if (s_fail) break;
      const uint32_t nr = s_hdr[1];
      uint32_t q0 = s_hdr[2], done = 0; // varints decoded of this entry's 2 * nr
      while (done < 2 * nr) {
        // tile [q0, q0 + LPD_NT * LPD_B) staged in LDS: lane t looks at bytes q0 + t * B .. + B
        const uint32_t te = q0 + LPD_NT * LPD_B < L ? q0 + LPD_NT * LPD_B : L;
        const uint64_t abs0 = (uint64_t)(ub + q0);
        const uint32_t sh = (uint32_t)(abs0 & 3), nw = (te - q0 + sh + 3) >> 2;
        __syncthreads();
        for (uint32_t q = t; q < nw; q += LPD_NT) tileb[q] = ((const uint32_t *)(abs0 - sh))[q];
        __syncthreads();
        auto tb = [&](uint32_t q) -> uint32_t { // update byte q in [q0, te)
          const uint32_t o = q - q0 + sh;
          return (tileb[o >> 2] >> ((o & 3) * 8)) & 0xFF;
        };
        const uint32_t b0 = q0 + t * LPD_B;
        uint32_t tm = 0; // terminator mask of my bytes
        for (uint32_t j = 0; j < LPD_B; j++)
          if (b0 + j < te && tb(b0 + j) < 0x80) tm |= 1u << j;
        uint32_t tot;
        const uint32_t pre = bscan_sum<LPD_NT>(__popc(tm), ws, tot);
        if (tot == 0) { // no terminator in the tile: EOS or an over-long varint
          if (t == 0) s_fail = 1;
          __syncthreads();
          break;
        }
        const uint32_t need = 2 * nr - done, take = tot < need ? tot : need;
        uint32_t lastend = 0;
        // varint j (0-based within the tile) starts after terminator j - 1 (or at q0); the
        // ones taken end inside the tile
        for (uint32_t j = 0; j < LPD_B; j++) {
          if (b0 + j >= te) break;
          const bool starts = (b0 + j == q0) || (j ? (tm >> (j - 1)) & 1 : (b0 > q0 && tb(b0 - 1) < 0x80));
          const uint32_t ordv = pre + __popc(tm & ((1u << j) - 1)); // terminators before this byte
          if (starts && ordv < take) {
            uint32_t x = 0, shv = 0, q = b0 + j;
            bool ok = true;
            for (;;) { // read_var_u32 (varint.rs:244-260)
              const uint32_t byte = tb(q++);
              x |= (byte & 0x7f) << (shv & 31);
              shv += 7;
              if (byte < 0x80) break;
              if (shv > 70) {
                ok = false;
                break;
              }
            }
            if (!ok) {
              s_fail = 1;
            } else if (!big) {
              const uint32_t gi = done + ordv, kr = rtot + gi / 2;
              if (gi & 1) rw[3 * kr + 1] = x; // length (start + length below)
              else {
                rw[3 * kr] = x;
                rw[3 * kr + 2] = e;
              }
            }
          }
          if (((tm >> j) & 1) && ordv + 1 == take) lastend = b0 + j + 1;
        }
        if (lastend) s_hdr[3] = lastend;
        __syncthreads();
        done += take;
        q0 = s_hdr[3];
        __syncthreads();
        if (s_fail) break;
      }
      __syncthreads();
      if (s_fail) break;
      if (t == 0) s_hdr[2] = q0;
      // start + length -> end (u32 overflow: update.rs id_set E_PANIC)
      if (!big)
        for (uint32_t kr = t; kr < nr; kr += LPD_NT) {
          const uint32_t st = rw[3 * (rtot + kr)], ln = rw[3 * (rtot + kr) + 1];
          if ((uint64_t)st + ln > 0xFFFFFFFFull) s_fail = 1;
          rw[3 * (rtot + kr) + 1] = st + ln;
        }
      rtot += nr;
      __syncthreads();
      if (s_fail) break;
    }
    __syncthreads();
    if (t == 0) {
      if (s_fail) {
        lp_fail(a, k);
      } else {
        m[LPM_NE] = nds;
        m[LPM_NR] = rtot;
        if (!big) { // table codes (OvfFill::on_ds_done)
          if (nds == 1) ov[1] = 0x80000000u;
          else if (nds >= 2) ds_order_packed(s_cl, nds, ov + nds, 0);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ k_lp_final
// lane per update: the record (rec_pack), or the exact walker's list
__global__ void __launch_bounds__(256) k_lp_final(LpArgs a) {
  const uint32_t n = a.g[LPG_N];
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
    const uint32_t *m = lp_meta(a, k);
    const uint64_t u = m[LPM_U] | ((uint64_t)m[LPM_U + 1] << 32);
    const uint32_t fl = m[LPM_FLAGS];
    if (fl & LPF_FALLBACK) {
      const uint32_t q = atomicAdd(&a.huge[1], 1u);
      a.fb[q] = u;
      continue;
    }
    RegSink s;
    s.nb = m[LPM_NB];
    s.ne = m[LPM_NE];
    s.nr = m[LPM_NR];
    s.unsupported = (fl & LPF_UNSUP) != 0;
    s.big_ds = s.ne > DS_SMALL;
    s.misorder = (fl & LPF_ORDER) != 0;
    const uint32_t *ov = a.ovf + m[LPM_OVF];
    if (s.nb) {
      s.b_client = ov[0];
      s.b_clock = ov[1];
      s.b_len = ov[2];
      s.b_pos = ov[3];
      s.b_meta = ov[4];
    }
    const uint32_t *ev = ov + 5 * s.nb;
    if (s.ne && !s.big_ds) {
      s.e_client = ev[0];
      const uint32_t *rv = ev + 2 * s.ne;
      if (s.nr > 0) {
        s.r0s = rv[0];
        s.r0e = rv[1];
      }
      if (s.nr > 1) {
        s.r1s = rv[3];
        s.r1e = rv[4];
      }
    }
    uint32_t w0, w1, w2, w3, w4, w5;
    rec_pack(s, 0, w0, w1, w2, w3, w4, w5);
    if (((w0 >> 10) & 3) == REC_COMPLEX && !s.big_ds) {
      w0 |= REC_OVF;
      w4 = m[LPM_OVF];
      w5 = k + 1; // the update's LP entry (single-update documents: grid paths)
      if (!(fl & (LPF_MSEC | LPF_SKIP | LPF_ZGC | LPF_PANIC | LPF_UNSUP)) && s.ne <= 1) w0 |= REC_LONG;
    }
    uint2 *o = (uint2 *)(a.rec + u * REC_WORDS);
    o[0] = make_uint2(w0, w1);
    o[1] = make_uint2(w2, w3);
    o[2] = make_uint2(w4, w5);
  }
}

void launch_long_decode(const LpArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k_lp_plan, dim3(1), dim3(1024), 0, s, a);
  const uint32_t gch = a.ccap < 1024 ? a.ccap : 1024;
  hipLaunchKernelGGL(k_lp_ext, dim3(2048), dim3(LPE_NT), 0, s, a);
  hipLaunchKernelGGL(k_lp_chunk, dim3(gch ? gch : 1), dim3(LP_NT), 0, s, a);
  hipLaunchKernelGGL(k_lp_stitch, dim3(1024), dim3(64), 0, s, a);
  hipLaunchKernelGGL(k_lp_expand, dim3(1024), dim3(LPX_NT), 0, s, a);
  launch_scan_u64(a.blen, a.sblen, a.ocap, a.scan_tmp, s, a.g + LPG_ORDS);
  hipLaunchKernelGGL(k_lp_clock, dim3(1024), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_lp_ds, dim3(2048), dim3(LPD_NT), 0, s, a);
  hipLaunchKernelGGL(k_lp_final, dim3(16), dim3(256), 0, s, a);
}

// ================================================================== single long update documents
// A document that is one update of one client section (REC_LONG: no Skips, no zero-length GC
// blocks, no panicking splits, <= 1 DeleteSet entry) is, for merge_updates_v1 (update.rs:537-704
// with one decoder), that section's blocks re-encoded in order behind one header and the union
// of its deleted ranges; for diff_updates_v1 (update.rs:490-535) the blocks from the first one
// past the remote clock (spliced by the offset) and the DeleteSet as decoded; for the state
// vector (update.rs:107-114) the last block's end.  Every block and range is a lane: sizes, a
// scan, then the writes -- instead of one workgroup (tiled kernel) or one lane (planners).

// merge: documents on path 2 that are one REC_LONG update
__global__ void __launch_bounds__(256) k_ls_find(BatchIn b, const uint8_t *path, uint32_t *list) {
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d >= b.n_docs || path[d] != 2) return;
  const uint64_t u = b.doc_upd[d];
  if (b.doc_upd[d + 1] - u != 1) return;
  const uint32_t *w = b.rec + u * REC_WORDS;
  const uint32_t w0 = w[0];
  if (!(w0 & REC_LONG) || (w0 & (0xFF | REC_SLOW)) || !(w0 & REC_OVF)) return;
  const uint32_t k = atomicAdd(&list[0], 1u);
  if (k >= LS_LIST) return;
  uint32_t *e = list + 4 + LS_EW * k;
  e[0] = d;
  e[1] = (uint32_t)u;
  e[2] = (uint32_t)(u >> 32);
  e[3] = (uint32_t)(b.upd_off[u + 1] - b.upd_off[u]);
  e[4] = w[1];
  e[5] = w[2];
  e[6] = w[3];
  e[7] = w[4];
}
void launch_ls_find(const BatchIn &b, const uint8_t *path, uint32_t *list, hipStream_t s) {
  if (!b.n_docs) return;
  hipLaunchKernelGGL(k_ls_find, dim3((b.n_docs + 255) / 256), dim3(256), 0, s, b, path, list);
}

// diff / SV: documents of >= min_len bytes -> the long-update list (huge) for the parallel parse
__global__ void __launch_bounds__(256) k_ls_list_diff(const uint64_t *upd_off, const uint8_t *pre_status,
                                                      uint32_t n_docs, uint32_t min_len, uint32_t *huge) {
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d >= n_docs || (pre_status && pre_status[d])) return;
  const uint64_t L = upd_off[d + 1] - upd_off[d];
  if (L < min_len || L >= LP_UNST) return;
  const uint32_t k = atomicAdd(&huge[0], 1u);
  if (k < HUGE_LIST) ((uint64_t *)(huge + 4))[k] = d;
}
void launch_ls_list_diff(const uint64_t *upd_off, const uint8_t *pre_status, uint32_t n_docs, uint32_t min_len,
                         uint32_t *huge, hipStream_t s) {
  if (!n_docs) return;
  hipLaunchKernelGGL(k_ls_list_diff, dim3((n_docs + 255) / 256), dim3(256), 0, s, upd_off, pre_status, n_docs,
                     min_len, huge);
}
// lane per parsed long update (update index = document): REC_LONG records -> list entries
__global__ void __launch_bounds__(256) k_ls_collect(LpArgs a, uint32_t *list) {
  const uint32_t n = a.g[LPG_N];
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
    const uint32_t *m = lp_meta(a, k);
    if (m[LPM_FLAGS] & LPF_FALLBACK) continue;
    const uint64_t u = m[LPM_U] | ((uint64_t)m[LPM_U + 1] << 32);
    const uint32_t *w = a.rec + u * REC_WORDS;
    const uint32_t w0 = w[0];
    if (!(w0 & REC_LONG) || (w0 & (0xFF | REC_SLOW)) || !(w0 & REC_OVF)) continue;
    const uint32_t q = atomicAdd(&list[0], 1u);
    if (q >= LS_LIST) continue;
    uint32_t *e = list + 4 + LS_EW * q;
    e[0] = (uint32_t)u;
    e[1] = (uint32_t)u;
    e[2] = (uint32_t)(u >> 32);
    e[3] = m[LPM_L];
    e[4] = w[1];
    e[5] = w[2];
    e[6] = w[3];
    e[7] = w[4];
  }
}
void launch_ls_collect(const LpArgs &a, uint32_t *list, hipStream_t s) {
  hipLaunchKernelGGL(k_ls_collect, dim3(16), dim3(256), 0, s, a, list);
}

__device__ __forceinline__ const uint32_t *ls_rv(const LsArgs &a) { return a.ov + 5 * a.NB + 2 * a.NE; }
__device__ __forceinline__ const uint8_t *ls_ub(const LsArgs &a) { return a.bytes + a.upd_off[a.u]; }

// one lane: state vector lookup / first diff block / headers
__global__ void k_ls_prep(LsArgs a) {
  if (threadIdx.x) return;
  uint32_t *g = a.g;
  for (uint32_t q = 0; q < LSG_WORDS; q++) g[q] = 0;
  const uint32_t NB = a.NB;
  const uint32_t client = NB ? a.ov[0] : 0u;
  g[LSG_CLIENT] = client;
  if (a.mode == 0) { // merge
    g[LSG_HDR] = NB ? varlen(1) + varlen(NB) + varlen(client) + varlen(a.ov[1]) : 1u;
    if (a.NE == 1 && a.NR == 0) g[LSG_BAD] = 1; // an entry without ranges: tiled kernel
    return;
  }
  if (a.mode == 2) { // Update::state_vector: the last stored block's end (+1 for GC)
    if (!NB) {
      g[LSG_BAD] = 1; // an empty section panics in yrs: the planner reports it
      return;
    }
    const uint32_t *r = a.ov + 5 * (NB - 1);
    const uint64_t end = (uint64_t)r[1] + r[2] + ((r[4] & 3) == BK_GC ? 1 : 0);
    if (end > 0xFFFFFFFFull) {
      g[LSG_BAD] = 1;
      return;
    }
    g[LSG_END] = (uint32_t)end;
    g[LSG_HDR] = varlen(1) + varlen(client) + varlen(end);
    return;
  }
  // diff: StateVector::decode (state_vector.rs:107-120), last insert of a client wins
  const uint64_t s0 = a.sv_off[a.d], s1 = a.sv_end ? a.sv_end[a.d] : a.sv_off[a.d + 1];
  Cur c{a.sv + s0, (uint32_t)(s1 - s0), 0};
  bool cn;
  uint32_t n, rc = 0;
  if (s1 - s0 >= (1ull << 31) || rd_var_u32(c, n, cn) || n > c.n) {
    g[LSG_BAD] = 1;
    return;
  }
  for (uint32_t q = 0; q < n; q++) {
    uint64_t cl;
    uint32_t ck;
    if (rd_var_u64(c, cl, cn) || rd_var_u32(c, ck, cn)) {
      g[LSG_BAD] = 1;
      return;
    }
    if (cl == client) rc = ck;
  }
  // first block past the remote clock (the blocks are contiguous: their ends increase)
  uint32_t lo = 0, hi = NB;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) / 2;
    const uint32_t *r = a.ov + 5 * mid;
    if ((uint64_t)r[1] + r[2] > rc) hi = mid;
    else lo = mid + 1;
  }
  const uint32_t k0 = lo;
  const uint32_t off = k0 < NB && rc > a.ov[5 * k0 + 1] ? rc - a.ov[5 * k0 + 1] : 0u;
  g[LSG_K0] = k0;
  g[LSG_OFF] = off;
  g[LSG_CLOCK] = k0 < NB ? a.ov[5 * k0 + 1] + off : 0u;
  g[LSG_HDR] = k0 < NB ? varlen(1) + varlen(NB - k0) + varlen(client) + varlen(g[LSG_CLOCK]) : 1u;
}

// The bytes of blocks [i0, i0 + 256) (consecutive in the update: one section) staged in LDS, at
// most LS_STAGE of them; returns the pointer p with p[q - s0] = update byte q for q in [s0, s1)
// (positions are passed relative to s0: a pointer below the LDS array would leave the LDS
// aperture once cast to a flat address)
constexpr uint32_t LS_STAGE = 16384;
__device__ __forceinline__ const uint8_t *ls_stage(const LsArgs &a, const uint8_t *ub, uint32_t i0, uint32_t *stage,
                                                   uint32_t &s0, uint32_t &s1) {
  s0 = s1 = 0;
  if (i0 >= a.NB) return ub;
  const uint32_t last = i0 + 255 < a.NB ? i0 + 255 : a.NB - 1;
  s0 = a.ov[5 * i0 + 3];
  s1 = a.ov[5 * last + 3] + (a.ov[5 * last + 4] >> 8);
  if (s1 - s0 > LS_STAGE) s1 = s0 + LS_STAGE;
  const uint64_t abs0 = (uint64_t)(ub + s0);
  const uint32_t sh = (uint32_t)(abs0 & 3), nw = (s1 - s0 + sh + 3) >> 2;
  const uint32_t *src = (const uint32_t *)(abs0 - sh);
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < nw; q += 256) stage[q] = src[q];
  __syncthreads();
  return (const uint8_t *)stage + sh; // p[q - s0] = update byte q
}

// lane per block and per range: sizes and checks
__global__ void __launch_bounds__(256) k_ls_size(LsArgs a) {
  __shared__ __align__(16) uint32_t stage[LS_STAGE / 4 + 4];
  ym_set_grammar(a.v1x);
  uint32_t *g = a.g;
  const uint32_t n = a.NB > a.NR ? a.NB : a.NR;
  const uint32_t k0 = g[LSG_K0], off = g[LSG_OFF];
  const uint32_t *rv = ls_rv(a);
  const uint8_t *ub = ls_ub(a);
  uint32_t bad = 0;
  for (uint32_t i0 = blockIdx.x * 256; i0 < n; i0 += gridDim.x * 256) {
    const uint32_t i = i0 + threadIdx.x;
    uint32_t s0, s1;
    const uint8_t *lb = a.mode == 2 ? ub : ls_stage(a, ub, i0, stage, s0, s1);
    if (i < a.NB) {
      const uint32_t *r = a.ov + 5 * i;
      const bool in_lds = r[3] >= s0 && r[3] + (r[4] >> 8) <= s1;
      const uint8_t *bp = in_lds ? lb : ub;
      const uint32_t bn = in_lds ? a.L - s0 : a.L, bq = in_lds ? r[3] - s0 : r[3];
      uint64_t sz = 0;
      if (a.mode == 1 && i < k0) {
        sz = 0;
      } else if (a.mode == 1 && i == k0 && off) {
        Counter cn;
        if (emit_block(bp, bn, bq, r[0], r[1], r[2], off, cn)) bad = 1;
        sz = cn.n;
      } else {
        sz = canon_size(bp, bn, bq, r[0], r[1], r[2], r[4]);
      }
      a.bsz[i] = sz;
    }
    if (i < a.NR) {
      const uint32_t st = rv[3 * i], en = rv[3 * i + 1];
      const uint32_t pe = i ? rv[3 * (i - 1) + 1] : 0u;
      uint64_t sz = 0;
      if (a.mode == 0) { // IdRange::squash (id_set.rs:129-164) of sorted, non-overlapping ranges:
        // adjacent ranges join into runs; here 1 per run start, scanned into run indices
        if (en <= st || (i && pe > st)) bad = 1;
        sz = i == 0 || st > pe;
      } else { // encoded as decoded when squashed (id_set.rs:166-187, 256-266)
        if (i && st < pe) bad = 1;
        sz = varlen(st) + varlen(en - st);
      }
      a.rsz[i] = sz;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    bad |= __shfl_xor(bad, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (bad) atomicOr(&g[LSG_BAD], 1u);
  }
}

__device__ __forceinline__ uint64_t ls_payload(const LsArgs &a, const uint32_t *g) {
  const uint64_t body = a.mode == 2 ? 0 : a.boff[a.NB];
  const uint32_t k = a.mode == 0 ? (uint32_t)a.roff[a.NR] : a.NR; // merge: runs
  const uint64_t rb = a.mode == 0 ? a.roff2[a.NR] : a.roff[a.NR];  // range bytes
  const uint64_t ds = a.mode == 2 ? 0 : a.NE == 0 ? 1 : varlen(1) + varlen(a.ov[5 * a.NB]) + varlen(k) + rb;
  return g[LSG_HDR] + body + ds;
}
__device__ __forceinline__ uint64_t ls_framed(const LsArgs &a, uint64_t p) {
  return a.frame ? 2 + varlen(p) + p : p;
}

// one lane: totals; merge: the slot's capacity; diff / SV: size, status, done (planners skip it)
__global__ void k_ls_total(LsArgs a) {
  if (threadIdx.x) return;
  uint32_t *g = a.g;
  if (g[LSG_BAD]) return; // merge: stays on path 2; diff / SV: the planners take it
  const uint64_t p = ls_payload(a, g);
  if (a.mode == 0) {
    const uint64_t slot = 2 * a.upd_off[a.u] + 64ull * a.d;
    if (p > 2ull * a.L + 64) {
      g[LSG_BAD] = 1;
      return;
    }
    a.out_start[a.d] = slot;
    a.out_len[a.d] = p;
    a.status[a.d] = 0;
    a.path[a.d] = 0; // written by k_ls_write (next on the stream): the tiled kernel skips it
    atomicAdd(&a.npath[15], 1u);
  } else {
    a.size[a.d] = ls_framed(a, p);
    a.status[a.d] = 0;
    a.path[a.d] = 0; // (ps.big)
    a.done[a.d] = 1;
  }
}

__global__ void __launch_bounds__(256) k_ls_write(LsArgs a) {
  __shared__ __align__(16) uint32_t stage[LS_STAGE / 4 + 4];
  ym_set_grammar(a.v1x);
  const uint32_t *g = a.g;
  if (g[LSG_BAD]) return;
  uint8_t *base = a.mode == 0 ? a.out + 2 * a.upd_off[a.u] + 64ull * a.d : a.out + a.pack_off[a.d];
  const uint64_t p = ls_payload(a, g);
  if (a.frame) base += 2 + varlen(p);
  const uint32_t client = g[LSG_CLIENT];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (a.frame) { // y-sync [MSG_SYNC, SyncStep2 | SyncStep1, varbuf] (protocol.rs:219-233)
      Writer w{base - 2 - varlen(p), 0};
      w.u8(0);
      w.u8(a.frame == 1 ? 1 : 0);
      w_var(w, p);
    }
    Writer w{base, 0};
    if (a.mode == 2) {
      w_var(w, 1);
      w_var(w, client);
      w_var(w, g[LSG_END]);
      return;
    }
    const uint32_t k0 = a.mode == 1 ? g[LSG_K0] : 0u;
    if (k0 < a.NB) {
      w_var(w, 1);
      w_var(w, a.NB - k0);
      w_var(w, client);
      w_var(w, a.mode == 1 ? g[LSG_CLOCK] : a.ov[1]);
    } else {
      w_var(w, 0);
    }
    Writer v{base + g[LSG_HDR] + a.boff[a.NB], 0};
    if (a.NE == 0) {
      w_var(v, 0);
    } else {
      w_var(v, 1);
      w_var(v, a.ov[5 * a.NB]);
      w_var(v, a.mode == 0 ? (uint32_t)a.roff[a.NR] : a.NR);
    }
  }
  if (a.mode == 2) return;
  const uint32_t n = a.NB > a.NR ? a.NB : a.NR;
  const uint32_t k0 = a.mode == 1 ? g[LSG_K0] : 0u, off = a.mode == 1 ? g[LSG_OFF] : 0u;
  const uint32_t *rv = ls_rv(a);
  const uint8_t *ub = ls_ub(a);
  uint8_t *blocks = base + g[LSG_HDR];
  uint8_t *ds = blocks + a.boff[a.NB] +
                (a.NE == 0 ? 1 : varlen(1) + varlen(a.ov[5 * a.NB]) + varlen(a.mode == 0 ? (uint32_t)a.roff[a.NR] : a.NR));
  for (uint32_t i0 = blockIdx.x * 256; i0 < n; i0 += gridDim.x * 256) {
    const uint32_t i = i0 + threadIdx.x;
    uint32_t s0, s1;
    const uint8_t *lb = ls_stage(a, ub, i0, stage, s0, s1);
    if (i < a.NB && i >= k0) {
      const uint32_t *r = a.ov + 5 * i;
      const bool in_lds = r[3] >= s0 && r[3] + (r[4] >> 8) <= s1;
      const uint8_t *bp = in_lds ? lb : ub;
      const uint32_t bn = in_lds ? a.L - s0 : a.L, bq = in_lds ? r[3] - s0 : r[3];
      Writer w{blocks + a.boff[i], 0};
      const uint32_t o = i == k0 ? off : 0u;
      if (o || ((r[4] & 4) && !(r[4] & 8))) {
        emit_block(bp, bn, bq, r[0], r[1], r[2], o, w);
      } else {
        const uint8_t *src = bp + bq;
        const uint32_t nb = r[4] >> 8;
        for (uint32_t q = 0; q < nb; q++) w.p[q] = src[q];
      }
    }
    if (a.mode == 0) { // run i (< the run count)
      if (i < a.NR && i < a.roff[a.NR]) {
        Writer w{ds + a.roff2[i], 0};
        w_var(w, a.rstart[i]);
        w_var(w, a.rend[i] - a.rstart[i]);
      }
    } else if (i < a.NR) {
      const uint32_t st = rv[3 * i];
      Writer w{ds + a.roff[i], 0};
      w_var(w, st);
      w_var(w, rv[3 * i + 1] - st);
    }
  }
}

// merge: lane per range -> the runs' starts and ends at their run indices (run starts scanned),
// then lane per run -> its encoded size
__global__ void __launch_bounds__(256) k_ls_runs(LsArgs a) {
  if (a.g[LSG_BAD]) return;
  const uint32_t *rv = ls_rv(a);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < a.NR; i += gridDim.x * 256) {
    const uint32_t st = rv[3 * i], en = rv[3 * i + 1];
    const bool f = i == 0 || st > rv[3 * (i - 1) + 1], last = i + 1 == a.NR || rv[3 * (i + 1)] > en;
    if (f) a.rstart[a.roff[i]] = st;
    if (last) a.rend[a.roff[i] + (f ? 1 : 0) - 1] = en;
  }
}
__global__ void __launch_bounds__(256) k_ls_runsize(LsArgs a) {
  const uint32_t K = a.g[LSG_BAD] ? 0u : (uint32_t)a.roff[a.NR];
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < a.NR; k += gridDim.x * 256)
    a.rsz2[k] = k < K ? varlen(a.rstart[k]) + varlen(a.rend[k] - a.rstart[k]) : 0u;
}

void launch_ls_doc(const LsArgs &a, int phase, hipStream_t s) {
  const uint32_t n = a.NB > a.NR ? a.NB : a.NR;
  const uint32_t gr = n ? (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024 : 1;
  if (phase == 0) {
    hipLaunchKernelGGL(k_ls_prep, dim3(1), dim3(64), 0, s, a);
    if (a.mode != 2) {
      hipLaunchKernelGGL(k_ls_size, dim3(gr), dim3(256), 0, s, a);
      launch_scan_u64(a.bsz, a.boff, a.NB, a.scan_tmp, s);
      launch_scan_u64(a.rsz, a.roff, a.NR, a.scan_tmp, s);
      if (a.mode == 0 && a.NR) {
        const uint32_t gn = (a.NR + 255) / 256 < 1024 ? (a.NR + 255) / 256 : 1024;
        hipLaunchKernelGGL(k_ls_runs, dim3(gn), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_ls_runsize, dim3(gn), dim3(256), 0, s, a);
        launch_scan_u64(a.rsz2, a.roff2, a.NR, a.scan_tmp, s);
      } else if (a.mode == 0) {
        launch_scan_u64(a.rsz2, a.roff2, 0, a.scan_tmp, s); // (roff2[0] = 0)
      }
    }
    hipLaunchKernelGGL(k_ls_total, dim3(1), dim3(64), 0, s, a);
    if (a.mode == 0) hipLaunchKernelGGL(k_ls_write, dim3(gr), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(k_ls_write, dim3(gr), dim3(256), 0, s, a);
  }
}

} // namespace ym
