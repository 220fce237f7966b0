// ymerge_fast.hip — parallel merge_updates_v1: one workgroup per document, LDS-resident.
//
// Stages (all inside one launch, one document per workgroup):
//   0 k_decode: (separate launch, one lane per update over the batch) LDS-staged
//               walk of every update -> one fixed-size record per update
//   1 gather  : lane-per-update record loads, counts -> block scan -> SoA block /
//               DeleteSet records at their scanned positions (rare multi-block
//               updates are walked again over HBM)
//   3 sort    : blocks by (client desc, clock asc, input order) — LDS bitonic,
//               skipped when already ordered
//   4 squash  : segmented max-scan of block ends -> keep / gap(Skip) / violation.
//               Fast-path precondition: every block starts at or
//               after the running end, or is fully covered with a later start, or
//               is a byte-identical duplicate.  Otherwise the document is handed to
//               the exact per-document engine (ymerge_seq.hip).
//   5 DS union: entries sorted by (client, first occurrence) -> yrs' hashbrown
//               client order; ranges sorted by (client, start) -> segmented union
//               (join overlapping or adjacent, id_set.rs:129-164)
//   6 encode  : prefix sums over output sizes; each lane writes its pieces into the
//               document's output slot (canonical re-encode only where the input was
//               not canonical).
#include "ycodec.h"
#include "ykernels.h"
#include "ywalk.h"
#include "ysm.h"
#include "ylds.h"
#include "yblock.h"

namespace ym {

// ------------------------------------------------------------------ LDS layout
// [block records][DS records][misc] then a union of two phase-local regions:
//   phase 3/4/6 (blocks): sort keys, classify flags, per-position output offsets
//   phase 5 (DeleteSet): sort keys, union flags/offsets, per-client tables
struct FastLayout {
  uint32_t bc, bk, bl, bp, bm, ec, et, rs, re, ri;
  uint32_t skey, sval;
  uint32_t dkey, dval, cend, coff, chead, dcl, dfirst, dord, dnc, dbeg, doff, dtab;
  uint32_t misc, stage, total;
};
constexpr uint32_t FAST_BCAP = 1024;   // blocks per document on the fast path (caps.b_cap)
constexpr uint32_t BMAP_WORDS = 1024;
constexpr uint32_t OVF_BATCH = 16;     // overflow words of a DeleteSet-only update loaded at once  // DeleteSet union bitmap (32768 clocks over all clients)
constexpr uint32_t DCAP = 64;          // distinct DeleteSet clients per document on the fast path
constexpr uint32_t DTAB_SLOTS = 256;   // LDS hash table for them
constexpr uint32_t BTAB = 64; // client table of the counting sort (<= 8 distinct clients used)
// LDS staging of the block section (6b): the phase-local union is free while it is written;
// it is grown to at least this size (total stays under 160 KB / 3 workgroups per CU)
constexpr uint32_t STAGE_MIN = 20 * 1024;
__host__ __device__ inline FastLayout fast_layout(const FastCaps &c) {
  FastLayout L;
  uint32_t o = 0;
  auto take = [&](uint32_t bytes) {
    uint32_t r = o;
    o += (bytes + 15) & ~15u;
    return r;
  };
  const uint32_t BS = pow2ceil(c.b_cap), RS = pow2ceil(c.r_cap > c.e_cap ? c.r_cap : c.e_cap);
  L.bc = take(4 * c.b_cap);
  L.bk = take(4 * c.b_cap);
  L.bl = take(4 * c.b_cap);
  L.bp = take(4 * c.b_cap);
  L.bm = take(4 * c.b_cap);
  L.ec = take(4 * c.e_cap);
  L.et = take(4 * c.e_cap);
  L.rs = take(4 * c.r_cap);
  L.re = take(4 * c.r_cap);
  L.ri = take(4 * c.r_cap);
  L.misc = take(4 * 256 + 8 * BTAB);
  const uint32_t u0 = o;
  uint32_t end = o;
  L.skey = take(8 * BS);
  L.sval = take(4 * BS);
  if (o > end) end = o;
  o = u0;
  L.dkey = take(8 * RS);
  L.dval = take(4 * RS);
  L.cend = take(4 * (RS + 1));
  L.coff = take(4 * (RS + 1));
  L.chead = take(4 * (RS + 1));
  L.dcl = take(4 * (DCAP + 1)); // per distinct DeleteSet client (D <= DCAP)
  L.dfirst = take(4 * (DCAP + 1));
  L.dord = take(4 * (DCAP + 1));
  L.dnc = take(4 * (DCAP + 1));
  L.dbeg = take(4 * (DCAP + 1));
  L.doff = take(4 * (DCAP + 1));
  L.dtab = take(8 * (DTAB_SLOTS > RS ? DTAB_SLOTS : RS)); // client table, then range sort keys (NR)
  if (o > end) end = o;
  L.stage = u0;
  if (u0 + STAGE_MIN > end) end = u0 + STAGE_MIN;
  L.total = end;
  return L;
}

// ------------------------------------------------------------------ k_decode
// overflow words past a workgroup's DEC_OVF: from the long-update region's 64-bit bump
// (huge[2..3]); UINT32_MAX when that is full too
__device__ __forceinline__ uint32_t ovf_global(uint32_t *huge, uint32_t need, uint32_t huge_base, uint64_t huge_cap) {
  const uint64_t at = atomicAdd((unsigned long long *)(huge + 2), (unsigned long long)need);
  return at + need <= huge_cap ? huge_base + (uint32_t)at : 0xFFFFFFFFu;
}

// One lane per update over the whole batch (updates of all documents are one
// contiguous byte range): the workgroup stages its NT updates' bytes into LDS with
// coalesced dword loads, every lane decodes its own update (fast_walk, branch-free
// varints) and writes one REC_WORDS record.  Other shapes and malformed updates are
// marked REC_SLOW and walked exactly (ysm.h) by k_fast_merge, so this kernel keeps
// the fast walk's small register footprint.
// Decoding here, rather than inside the per-document workgroup, runs the latency-bound
// byte walk at full occupancy (16 KB LDS, no per-document phases holding registers).
// 8 workgroups per CU (8 waves per SIMD): <= 64 VGPRs and < 20 KB of LDS (the second-walk
// list keeps 16-bit lane / count fields)
__global__ void __launch_bounds__(DEC_NT, 8) k_decode(const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_upd,
                                                      uint32_t *rec, uint32_t *ovf, uint32_t *huge, uint32_t v1x,
                                                      uint32_t lp_min, uint32_t lp_direct, uint32_t huge_base,
                                                      uint64_t huge_cap) {
  __shared__ __align__(16) uint32_t stage[DEC_STAGE / 4 + 4];
  __shared__ uint32_t ovf_top, n_cx, n_sl;
  ym_set_grammar(v1x); // (fast_walk bails on every content it does not restate)
  __shared__ uint32_t cx_at[DEC_NT];
  __shared__ uint16_t cx_lane[DEC_NT], cx_nb[DEC_NT], cx_ne[DEC_NT];
  const uint64_t g0 = (uint64_t)blockIdx.x * DEC_NT;
  const uint32_t t = threadIdx.x;
  const uint64_t i = g0 + t;
  const uint64_t rl = n_upd - g0 < DEC_NT ? n_upd - g0 : DEC_NT;
  const uint64_t A = upd_off[g0], E = upd_off[g0 + rl];
  // 16-byte loads, all issued before the first LDS store (one HBM round trip per lane)
  const uint64_t sbase = A & ~15ull;
  uint64_t n16 = (E - sbase + 15) >> 4;
  if (n16 > DEC_STAGE / 16) n16 = DEC_STAGE / 16;
  const uint64_t nd = 4 * n16;
  {
    constexpr uint32_t PL = DEC_STAGE / 16 / DEC_NT;
    const uint4 *src = (const uint4 *)(bytes + sbase);
    uint4 v[PL];
#pragma unroll
    for (uint32_t j = 0; j < PL; j++)
      if (t + j * DEC_NT < n16) v[j] = src[t + j * DEC_NT];
#pragma unroll
    for (uint32_t j = 0; j < PL; j++)
      if (t + j * DEC_NT < n16) ((uint4 *)stage)[t + j * DEC_NT] = v[j];
  }
  if (t == 0) {
    ovf_top = 0;
    n_cx = 0;
    n_sl = 0;
  }
  __syncthreads();
  if (i < n_upd) {
    const uint64_t a0 = upd_off[i], a1 = upd_off[i + 1];
    const uint32_t ulen = (uint32_t)(a1 - a0);
    RegSinkT<false> s; // (sections checked by the second walk)
    s.nb = s.ne = s.nr = 0;
    s.unsupported = s.big_ds = false;
    s.ubase = 0;
    const bool staged = a1 - sbase <= 4 * nd;
    // (an update of >= lp_direct bytes skips the lane walk: one lane stepping through KBs of
    // blocks, twice for the overflow words, held the whole workgroup for ~1 ms)
    const int e = staged && ulen < lp_direct ? fast_walk(stage, (uint32_t)(a0 - sbase), ulen, s) : -1;
    // a long update (or a medium one the fast walk cannot take): the parallel parse (ylong.hip)
    const bool lp_take = e < 0 && ulen >= lp_min;
    if (lp_take) {
      const uint32_t k = atomicAdd(&huge[0], 1u);
      if (k < HUGE_LIST) ((uint64_t *)(huge + 4))[k] = i;
    } else if (e < 0) { // a shape the fast walk does not restate, or past the stage:
      atomicAdd(&n_sl, 1u); // k_decode_exact (record REC_SLOW | REC_STAGED)
    }
    uint32_t w0 = lp_take ? REC_SLOW : REC_SLOW | REC_STAGED, w1 = 0, w2 = 0, w3 = 0, w4 = 0, w5 = 0;
    if (e >= 0) rec_pack(s, e, w0, w1, w2, w3, w4, w5);
    if (e == 0 && ((w0 >> 10) & 3) == REC_COMPLEX && !s.big_ds) {
      // multi-record update: its records go to this workgroup's overflow words (LDS bump
      // allocation), written by the second walk below; if they do not fit, k_fast_merge
      // walks the update again
      const uint32_t need = 5 * s.nb + 2 * s.ne + 3 * s.nr;
      const uint32_t off = need <= DEC_OVF ? atomicAdd(&ovf_top, need) : DEC_OVF;
      // no room in the workgroup's words: the long-update region's bump (huge[2..3])
      const uint32_t at = off + need <= DEC_OVF ? blockIdx.x * DEC_OVF + off
                                                : ovf_global(huge, need, huge_base, huge_cap);
      if (at == 0xFFFFFFFFu) { // none there either: k_decode_exact walks it
        w0 = REC_SLOW | REC_STAGED;
        atomicAdd(&n_sl, 1u);
      } else {
        w0 |= REC_OVF;
        w4 = at;
        const uint32_t q = atomicAdd(&n_cx, 1u);
        cx_lane[q] = t;
        cx_at[q] = at;
        cx_nb[q] = (uint16_t)s.nb; // a staged update is <= DEC_STAGE (16 KB): its counts are < 2^16
        cx_ne[q] = (uint16_t)s.ne;
      }
    }
    uint2 *o = (uint2 *)(rec + i * REC_WORDS);
    o[0] = make_uint2(w0, w1);
    o[1] = make_uint2(w2, w3);
    o[2] = make_uint2(w4, w5);
  }
  __syncthreads();
  // the staged updates the fast walk left: k_decode_exact walks them exactly over the same stage
  // (a kernel of its own: the exact walk's registers would halve this kernel's occupancy)
  if (t == 0 && n_sl) {
    const uint32_t k = atomicAdd(&huge[EXQ_COUNT], 1u);
    uint32_t *e = huge + EXQ_LIST + 2 * k;
    e[0] = blockIdx.x;
    e[1] = ovf_top; // (the exact walks continue the workgroup's overflow allocation)
  }
  // second walk of the multi-record updates, packed onto the first lanes: a wave runs it
  // only when it holds one of them (a few percent of an editor's updates), instead of every
  // wave whose lanes happen to include one
  for (uint32_t q = t; q < n_cx; q += DEC_NT) {
    const uint64_t j = g0 + cx_lane[q];
    const uint64_t a0 = upd_off[j], a1 = upd_off[j + 1];
    OvfFill f{ovf + cx_at[q], cx_nb[q], cx_ne[q], 0, 0, 0};
    fast_walk(stage, (uint32_t)(a0 - sbase), (uint32_t)(a1 - a0), f);
    if (f.misorder) rec[j * REC_WORDS] |= REC_ORDER; // (written by this workgroup before the barrier)
  }
}

// The workgroups of k_decode that left updates to the exact walk (listed with their overflow
// bump): k_decode's 16 KB stage again, and further stages from the first update still pending
// (the updates past the first stage).  The pending updates of a stage are walked exactly (ysm.h
// over the stage) one per wavefront, all 64 lanes in lockstep: the state-machine walk of 64
// different updates on 64 lanes diverges at every step (a tile of rich-content updates took
// ~17 ms that way), one walk in lockstep does not.  Records and overflow words are written as
// k_decode writes them (lane 0).
// EX_NT 256 (one wavefront per SIMD): the lockstep walk keeps its state in registers (at 1024
// threads its 128-VGPR budget spilled the walk's state to scratch on every step); EX_SPLIT
// workgroups share a tile, each walking the pending updates u of it with u % EX_SPLIT == its part
// (each stages on its own), and take overflow words from the tile's bump in the exact list (a
// global atomic)
constexpr uint32_t EX_NT = 256, EX_NW = EX_NT / 64, EX_SPLIT = 8;
template <bool LANE>
__global__ void __launch_bounds__(EX_NT) k_decode_exact(const uint8_t *bytes, const uint64_t *upd_off,
                                                       uint64_t n_upd, uint32_t *rec, uint32_t *ovf,
                                                       uint32_t *huge, uint32_t v1x, uint32_t huge_base,
                                                       uint64_t huge_cap, uint64_t *dbg) {
  __shared__ __align__(16) uint32_t stage[DEC_STAGE / 4 + 4];
  __shared__ uint32_t n_sl, n_go;
  __shared__ unsigned long long s_next, s_max;
  __shared__ uint16_t sl_lane[DEC_NT], go_lane[DEC_NT];
  ym_set_grammar(v1x);
  const uint32_t t = threadIdx.x, wv = t >> 6, lane = t & 63, ntiles = huge[EXQ_COUNT];
  constexpr uint32_t SPLIT = LANE ? 1 : EX_SPLIT; // (lane mode: a workgroup walks 256 pending updates at once)
  const uint32_t part = blockIdx.x % SPLIT, nslot = gridDim.x / SPLIT; // (grid: a multiple of SPLIT)
  for (uint32_t k = blockIdx.x / SPLIT; k < ntiles; k += nslot) {
    const uint32_t b = huge[EXQ_LIST + 2 * k];
    uint32_t *ovf_top = huge + EXQ_LIST + 2 * k + 1;
    const uint64_t g0 = (uint64_t)b * DEC_NT;
    const uint64_t rl = n_upd - g0 < DEC_NT ? n_upd - g0 : DEC_NT;
    const uint64_t A = upd_off[g0], E = upd_off[g0 + rl];
    const uint64_t tk0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t nround = 0;
    __syncthreads();
    if (t == 0) {
      n_sl = 0;
      s_max = 0;
    }
    __syncthreads();
    for (uint32_t u = part + SPLIT * t; u < rl; u += SPLIT * EX_NT) // this workgroup's share of the tile
      if ((rec[(g0 + u) * REC_WORDS] & (REC_SLOW | REC_STAGED)) == (REC_SLOW | REC_STAGED))
        sl_lane[atomicAdd(&n_sl, 1u)] = (uint16_t)u;
    __syncthreads();
    uint64_t sbase = A & ~15ull;
    for (uint32_t round = 0; round < DEC_NT; round++) { // (each round takes >= 1 pending update)
      uint64_t n16 = (E - sbase + 15) >> 4;
      if (n16 > DEC_STAGE / 16) n16 = DEC_STAGE / 16;
      const uint64_t wend = sbase + 16 * n16;
      __syncthreads();
      for (uint32_t q = t; q < n16; q += EX_NT) ((uint4 *)stage)[q] = ((const uint4 *)(bytes + sbase))[q];
      if (t == 0) {
        n_go = 0;
        s_next = ~0ull;
      }
      __syncthreads();
      // the pending updates inside this stage go; the first one past it starts the next stage
      for (uint32_t q = t; q < n_sl; q += EX_NT) {
        const uint32_t ul = sl_lane[q];
        if (ul == 0xFFFF) continue;
        const uint64_t a0 = upd_off[g0 + ul], a1 = upd_off[g0 + ul + 1];
        if (a0 >= sbase && a1 <= wend) {
          go_lane[atomicAdd(&n_go, 1u)] = (uint16_t)ul;
          sl_lane[q] = 0xFFFF;
        } else {
          atomicMin(&s_next, (unsigned long long)a0);
        }
      }
      __syncthreads();
      nround++;
      if (LANE) { // one update per lane (updates here are short: the long ones took the parallel parse)
        for (uint32_t q = t; q < n_go; q += EX_NT) {
          const uint64_t tw0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
          const uint64_t j = g0 + go_lane[q];
          const uint64_t a0 = upd_off[j], a1 = upd_off[j + 1];
          RegSink s;
          s.nb = s.ne = s.nr = 0;
          s.unsupported = s.big_ds = false;
          s.ubase = 0;
          const uint32_t base = (uint32_t)(a0 - sbase), len = (uint32_t)(a1 - a0);
          SCur c{(const uint8_t *)stage + base, len, 0, stage, base};
          const int e = smwalk_update(c, s);
          uint32_t w0, w1, w2, w3, w4, w5;
          rec_pack(s, e, w0, w1, w2, w3, w4, w5);
          if (e == 0 && ((w0 >> 10) & 3) == REC_COMPLEX && !s.big_ds) {
            const uint32_t need = 5 * s.nb + 2 * s.ne + 3 * s.nr;
            const uint32_t off = need <= DEC_OVF ? atomicAdd(ovf_top, need) : DEC_OVF;
            const uint32_t at = off + need <= DEC_OVF ? b * DEC_OVF + off : ovf_global(huge, need, huge_base, huge_cap);
            if (at != 0xFFFFFFFFu) { // second walk: the overflow words
              OvfFill f{ovf + at, s.nb, s.ne, 0, 0, 0};
              SCur c2{(const uint8_t *)stage + base, len, 0, stage, base};
              smwalk_update(c2, f);
              w0 |= REC_OVF;
              w4 = at;
            } else {
              w0 = REC_SLOW; // no overflow room: the merge kernels walk it
              w1 = w2 = w3 = w4 = w5 = 0;
            }
          }
          uint2 *o = (uint2 *)(rec + j * REC_WORDS);
          o[0] = make_uint2(w0, w1);
          o[1] = make_uint2(w2, w3);
          o[2] = make_uint2(w4, w5);
          if (dbg) atomicMax(&s_max, ((__builtin_amdgcn_s_memtime() - tw0) << 24) | (j & 0xFFFFFF));
        }
      } else
      for (uint32_t q = wv; q < n_go; q += EX_NW) { // one update per wavefront (uniform in it)
        const uint64_t tw0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
        const uint64_t j = g0 + go_lane[q];
        const uint64_t a0 = upd_off[j], a1 = upd_off[j + 1];
        RegSink s;
        s.nb = s.ne = s.nr = 0;
        s.unsupported = s.big_ds = false;
        s.ubase = 0;
        const uint32_t base = ym_uni((uint32_t)(a0 - sbase)), len = ym_uni((uint32_t)(a1 - a0));
        SCurU c;
        c.p = (const uint8_t *)stage + base;
        c.n = len;
        c.i = 0;
        c.w = stage;
        c.base = base;
        const int e = smwalk_update(c, s);
        uint32_t w0, w1, w2, w3, w4, w5;
        rec_pack(s, e, w0, w1, w2, w3, w4, w5);
        if (e == 0 && ((w0 >> 10) & 3) == REC_COMPLEX && !s.big_ds) {
          const uint32_t need = 5 * s.nb + 2 * s.ne + 3 * s.nr;
          uint32_t at = 0;
          if (lane == 0) {
            const uint32_t off = need <= DEC_OVF ? atomicAdd(ovf_top, need) : DEC_OVF;
            at = off + need <= DEC_OVF ? b * DEC_OVF + off : ovf_global(huge, need, huge_base, huge_cap);
          }
          at = (uint32_t)__builtin_amdgcn_readfirstlane((int)at);
          if (at != 0xFFFFFFFFu) { // second walk: the overflow words (lane 0 writes)
            OvfFill f{ovf + at, s.nb, s.ne, 0, 0, 0};
            f.on = lane == 0;
            SCurU c2;
            c2.p = (const uint8_t *)stage + base;
            c2.n = len;
            c2.i = 0;
            c2.w = stage;
            c2.base = base;
            smwalk_update(c2, f);
            w0 |= REC_OVF;
            w4 = at;
          } else {
            w0 = REC_SLOW; // no overflow room: the merge kernels walk it
            w1 = w2 = w3 = w4 = w5 = 0;
          }
        }
        if (lane == 0) {
          uint2 *o = (uint2 *)(rec + j * REC_WORDS);
          o[0] = make_uint2(w0, w1);
          o[1] = make_uint2(w2, w3);
          o[2] = make_uint2(w4, w5);
          if (dbg) atomicMax(&s_max, ((__builtin_amdgcn_s_memtime() - tw0) << 24) | (j & 0xFFFFFF));
        }
      }
      __syncthreads();
      if (s_next == ~0ull) break; // (uniform)
      sbase = s_next & ~15ull;
    }
    if (dbg && t == 0) { // diagnostic (env YMERGE_DECODE_DBG): tile, pending, rounds, cycles, slowest walk
      uint64_t *o = dbg + 8 * (size_t)k;
      if (part == 0) {
        o[0] = b;
        o[1] = n_sl;
        o[2] = nround;
        o[6] = E - A;
      }
      atomicMax((unsigned long long *)o + 3, (unsigned long long)(__builtin_amdgcn_s_memtime() - tk0));
      atomicMax((unsigned long long *)o + 7, s_max);
    }
  }
}

// The updates k_decode could not stage and listed (>= HUGE_MIN bytes): a wavefront each walks
// one through the LDS window of ylwin.h, all 64 lanes in lockstep (the exact walk of ysm.h, so
// records and errors are those of walk_record_hbm), and writes its record.  A multi-record
// update's overflow words come from a bump allocator over the tail of the overflow buffer
// (words huge_base.. huge_base + huge_cap); one that does not fit stays REC_SLOW.  The merge
// kernels then read records instead of walking the update over HBM, once per kernel, through
// a 64-byte register window (b4-update.bin: ~1 s -> a few ms).
__global__ void __launch_bounds__(64) k_decode_huge(const uint8_t *bytes, const uint64_t *upd_off, uint32_t *rec,
                                                   uint32_t *ovf, uint32_t *huge, const uint32_t *count,
                                                   const uint64_t *list, uint32_t huge_base, uint64_t huge_cap,
                                                   uint32_t v1x) {
  __shared__ __align__(16) uint32_t win[LW_BYTES / 4];
  ym_set_grammar(v1x);
  const uint32_t lane = threadIdx.x;
  const uint32_t n = *count < HUGE_LIST ? *count : HUGE_LIST;
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint64_t i = list[k];
    const uint64_t a0 = upd_off[i], a1 = upd_off[i + 1];
    const uint32_t ulen = (uint32_t)(a1 - a0);
    RegSink s;
    s.nb = s.ne = s.nr = 0;
    s.unsupported = s.big_ds = false;
    s.ubase = 0;
    LWin c;
    lw_init(c, bytes + a0, ulen, (lds_u32 *)win);
    const int e = smwalk_update(c, s);
    uint32_t w0, w1, w2, w3, w4, w5;
    rec_pack(s, e, w0, w1, w2, w3, w4, w5);
    bool write = true;
    if (e == 0 && ((w0 >> 10) & 3) == REC_COMPLEX && !s.big_ds) {
      const uint64_t need = 5ull * s.nb + 2ull * s.ne + 3ull * s.nr;
      uint64_t off = 0;
      // 64-bit bump (shared with the parallel parse): a request that does not fit still advances
      // it, but it cannot wrap onto words already handed out
      if (lane == 0) off = atomicAdd((unsigned long long *)(huge + 2), (unsigned long long)need);
      off = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(off >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)off);
      if (off + need <= huge_cap) {
        OvfFill f{ovf + huge_base + off, s.nb, s.ne, 0, 0, 0};
        LWin c2;
        lw_init(c2, bytes + a0, ulen, (lds_u32 *)win);
        smwalk_update(c2, f);
        w0 |= REC_OVF;
        w4 = huge_base + (uint32_t)off;
      } else {
        write = false; // no room: the record stays REC_SLOW
      }
    }
    if (write && lane == 0) {
      uint2 *o = (uint2 *)(rec + i * REC_WORDS);
      o[0] = make_uint2(w0, w1);
      o[1] = make_uint2(w2, w3);
      o[2] = make_uint2(w4, w5);
    }
  }
}

// k_decode, then the long updates it listed: the parallel parse (ylong.hip) when its scratch is
// given, the exact lockstep walk for the ones it leaves (errors, bounds); without it every listed
// update takes the exact walk
void launch_decode(const uint8_t *bytes, const uint64_t *upd_off, uint64_t n_updates, uint32_t *rec, uint32_t *ovf,
                   uint32_t *huge, uint32_t huge_cap, hipStream_t s, const LpArgs *lp, uint32_t v1x, uint64_t *dbg, uint32_t *h_probe) {
  if (!n_updates) return;
  const uint64_t nwg = (n_updates + DEC_NT - 1) / DEC_NT;
  hipMemsetAsync(huge, 0, 16, s);
  hipMemsetAsync(huge + EXQ_COUNT, 0, 4, s);
  const uint32_t lp_min = lp ? (lp->mid < LP_MIN_LEN ? lp->mid : LP_MIN_LEN) : LP_MIN_LEN;
  hipLaunchKernelGGL(k_decode, dim3((unsigned)nwg), dim3(DEC_NT), 0, s, bytes, upd_off, n_updates, rec, ovf, huge,
                     v1x, lp_min, lp ? LP_DIRECT_LEN : 0xFFFFFFFFu, (uint32_t)(nwg * DEC_OVF), (uint64_t)huge_cap);
  const uint32_t base = (uint32_t)(nwg * DEC_OVF);
  // (h_probe, pinned host words: one round trip reads whether k_decode listed anything for the
  // exact walk or the long-update path; a batch with neither skips their ~12 launches, ~60 us)
  bool any_exact = true, any_long = true;
  if (h_probe) {
    hipMemcpyAsync(h_probe, huge, 4, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(h_probe + 1, huge + EXQ_COUNT, 4, hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) == hipSuccess) {
      any_long = h_probe[0] != 0;
      any_exact = h_probe[1] != 0;
    }
  }
  static const bool lockstep = getenv("YMERGE_EXACT_LOCKSTEP") != nullptr; // (A/B: one update per wavefront)
  if (!any_exact) {
  } else if (lockstep)
    hipLaunchKernelGGL(k_decode_exact<false>, dim3((unsigned)(nwg < 512 ? nwg : 512) * EX_SPLIT), dim3(EX_NT), 0, s,
                       bytes, upd_off, n_updates, rec, ovf, huge, v1x, (uint32_t)(nwg * DEC_OVF), (uint64_t)huge_cap,
                       dbg);
  else // a workgroup per listed tile (the list is shorter than nwg)
    hipLaunchKernelGGL(k_decode_exact<true>, dim3((unsigned)(nwg < 65536 ? nwg : 65536)), dim3(EX_NT), 0, s,
                       bytes, upd_off, n_updates, rec, ovf, huge, v1x, (uint32_t)(nwg * DEC_OVF), (uint64_t)huge_cap,
                       dbg);
  if (!any_long) {
  } else if (lp) {
    LpArgs a = *lp;
    a.bytes = bytes;
    a.upd_off = upd_off;
    a.rec = rec;
    a.ovf = ovf;
    a.huge = huge;
    a.huge_base = base;
    a.huge_cap = huge_cap;
    launch_long_decode(a, s);
    hipLaunchKernelGGL(k_decode_huge, dim3(64), dim3(64), 0, s, bytes, upd_off, rec, ovf, huge,
                       (const uint32_t *)(huge + 1), (const uint64_t *)a.fb, base, (uint64_t)huge_cap, a.v1x);
  } else {
    hipLaunchKernelGGL(k_decode_huge, dim3(64), dim3(64), 0, s, bytes, upd_off, rec, ovf, huge, (const uint32_t *)huge,
                       (const uint64_t *)(huge + 4), base, (uint64_t)huge_cap, v1x);
  }
}

// ------------------------------------------------------------------ the kernel
// Diagnostic build only (STAMPS=true, env YMERGE_STAMPS): lane 0 records s_memtime at
// phase boundaries into o.stamps[doc * 16 + k]; never part of a timed run.
#define YM_STAMP(k)                                                                                \
  do {                                                                                             \
    if (STAMPS) {                                                                                  \
      __syncthreads();                                                                             \
      if (threadIdx.x == 0) o.stamps[(size_t)blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
    }                                                                                              \
  } while (0)

// k_fast_merge's single-update identity check (lane 0): the decoded record of update u (no
// error, flags, REC_SLOW) and, for a multi-record update, its overflow words
__device__ __noinline__ bool single_update_identity(const BatchIn &b, uint64_t u, uint32_t ulen) {
  const uint32_t *r = b.rec + (size_t)u * REC_WORDS;
  const uint32_t w0 = r[0];
  if (w0 & (0xFFu | REC_SLOW | REC_UNSUP | REC_BIGDS | REC_ORDER)) return false;
  const uint32_t shape = (w0 >> 10) & 3;
  uint64_t size = 0;
  if (shape == REC_EMPTY) {
    size = 2; // no section, no DeleteSet entry
  } else if (shape == REC_BLOCK) {
    const uint32_t meta = r[5], len = r[3];
    if ((meta & 12) || (meta & 3) == BK_SKIP || len == 0) return false;
    size = varlen(1) + varlen(1) + varlen(r[1]) + varlen(r[2]) + (meta >> 8) + 1;
  } else if (shape == REC_DS) {
    const uint32_t nr = (w0 >> 12) & 3;
    if (nr == 0 || r[3] <= r[2] || (nr == 2 && (r[5] <= r[4] || r[4] <= r[3]))) return false;
    size = 1 + 1 + varlen(r[1]) + varlen(nr) + varlen(r[2]) + varlen(r[3] - r[2]);
    if (nr == 2) size += varlen(r[4]) + varlen(r[5] - r[4]);
  } else {
    if (!(w0 & REC_OVF)) return false;
    const uint32_t nb = r[1], ne = r[2], nr = r[3];
    if (ne > 1 || nb > 4096 || nr > 4096) return false;
    const uint32_t *ov = b.ovf + r[4];
    uint32_t nsec = 0, cl = 0, nxt = 0, sec_nb = 0, sec_client = 0, sec_clock = 0;
    for (uint32_t k = 0; k < nb; k++) {
      const uint32_t c = ov[5 * k], ck = ov[5 * k + 1], len = ov[5 * k + 2], meta = ov[5 * k + 4];
      if ((meta & 12) || (meta & 3) == BK_SKIP || len == 0) return false;
      if (k == 0 || c != cl) { // a new section: strictly below the previous client
        if (k) {
          if (c > cl) return false;
          size += varlen(sec_nb) + varlen(sec_client) + varlen(sec_clock);
        }
        nsec++;
        sec_nb = 0;
        sec_client = c;
        sec_clock = ck;
      } else if (ck != nxt) {
        return false; // a gap (a Skip the record does not keep) or an overlap
      }
      sec_nb++;
      cl = c;
      nxt = ck + len;
      size += meta >> 8;
    }
    if (nb) size += varlen(sec_nb) + varlen(sec_client) + varlen(sec_clock);
    size += varlen(nsec);
    const uint32_t *ec = ov + 5 * nb, *rg = ec + 2 * ne;
    size += varlen(ne);
    if (ne == 1) {
      if (nr == 0 || ec[1] != 0x80000000u) return false;
      size += varlen(ec[0]) + varlen(nr);
      uint32_t prev_end = 0;
      for (uint32_t k = 0; k < nr; k++) {
        const uint32_t st = rg[3 * k], en = rg[3 * k + 1];
        if (en <= st || (k && st <= prev_end)) return false; // sorted, disjoint, not adjacent
        size += varlen(st) + varlen(en - st);
        prev_end = en;
      }
    } else if (nr) {
      return false;
    }
  }
  return size == ulen;
}

template <int NT, bool STAMPS>
__global__ void __launch_bounds__(NT, 3) k_fast_merge(BatchIn b, FastCaps caps, FastOut o) {
  ym_set_grammar(b.v1x);
  constexpr int PER = (int)(FAST_BCAP / NT); // sorted positions per lane (b_cap == FAST_BCAP)
  extern __shared__ __align__(16) uint8_t smem[];
  const FastLayout L = fast_layout(caps);
  const uint32_t d = blockIdx.x;
  if (d >= b.n_docs) return;
  if (b.only_path3 && o.path[d] != 3) return; // written by k_lean
  const uint32_t t = threadIdx.x;
  uint32_t *misc = (uint32_t *)(smem + L.misc);
  // misc[0] err key, [1] flags, [2..] scan workspace (NT/64*2+2 words), [64..] scalars
  uint32_t *ws = misc + 2;
  uint32_t *sc = misc + 64;

  const uint64_t u0 = b.doc_upd[d], u1 = b.doc_upd[d + 1];
  const uint32_t U = (uint32_t)(u1 - u0);
  const uint64_t B0 = b.upd_off[u0], B1 = b.upd_off[u1];
  const uint32_t nbytes = (uint32_t)(B1 - B0);
  const uint64_t slot = 2 * B0 + 64ull * d;
  const uint64_t cap = 2ull * nbytes + 64;
  const uint8_t *in = b.bytes + B0; // document bytes stay in HBM; lanes read them through WCur
  // path 1: exact engine (partial overlaps, comparator anomalies, ...); path 2: over the
  // LDS capacities only -> the tiled HBM-scratch kernel (ymerge_big.hip)
  auto handover = [&](uint8_t p = 1) {
    if (t == 0) {
      const uint32_t k = atomicAdd(&o.npath[p], 1u);
      if (p == 2 && o.big_list) o.big_list[k] = d; // (the tiled kernel's launch list)
      o.path[d] = p;
      o.status[d] = 0;
      o.out_len[d] = 0;
      o.out_start[d] = slot;
    }
  };
  // update indices are packed as (i << 8) into 31-bit LDS keys (first-occurrence order, first
  // error): documents with 2^23 or more updates go to the exact engine
  if (B1 - B0 >= (1ull << 31) || U >= (1u << 23)) {
    handover();
    return;
  }
  // One canonical update whose merge is itself (yrs merge_updates of a single update re-encodes
  // it: client sections in descending order, a client's blocks in queue order, nothing squashed,
  // the DeleteSet of <= 1 client re-encoded from sorted disjoint ranges): the bytes are copied.
  // The decoded record decides; the canonical size of what it holds must equal the update's
  // length, so a Skip, a dropped zero-length item or a non-canonical header (none of which the
  // record keeps) fails the check.  43 % of the reference corpus's documents are one update.
  if (U == 1 && caps.ident) {
    if (t == 0) misc[40] = single_update_identity(b, u0, nbytes) ? 1u : 0u;
    __syncthreads();
    if (misc[40]) {
      uint8_t *dst = o.out + slot;
      for (uint32_t q = 4 * t; q < nbytes; q += 4 * NT) {
        const uint32_t k = nbytes - q < 4 ? nbytes - q : 4;
        uint8_t v[4];
#pragma unroll
        for (uint32_t z = 0; z < 4; z++) v[z] = z < k ? in[q + z] : 0;
#pragma unroll
        for (uint32_t z = 0; z < 4; z++)
          if (z < k) dst[q + z] = v[z];
      }
      if (t == 0) {
        o.path[d] = 0;
        o.status[d] = 0;
        o.out_len[d] = nbytes;
        o.out_start[d] = slot;
      }
      return;
    }
    __syncthreads();
  }
  // Tiny documents (<= in_cap updates, <= u_cap bytes): one lane each in the lane-per-document
  // engine is cheaper than this workgroup's fixed phase sequence (C3: 2/3 of the documents;
  // measured 13.5 ms here vs 4.5 ms there for the 645k documents of <= 4 updates).
  if (U > 0 && U <= caps.in_cap && B1 - B0 <= caps.u_cap) {
    if (t == 0) atomicAdd(&o.npath[5], 1u);
    handover();
    return;
  }
  // More updates than blocks + DeleteSet entries fit: every update that is not empty adds a
  // block or an entry, so the document cannot fit (or is mostly empty updates, which the
  // tiled kernel merges as well): hand it over before decoding (C4: 2.5 ms of rounds that
  // ended in the same hand-over)
  if (U > caps.b_cap + caps.e_cap) {
    handover(2);
    return;
  }
  if (t == 0) {
    misc[0] = 0xFFFFFFFFu;
    misc[1] = 0;
  }
  YM_STAMP(0);
  uint32_t *bc = (uint32_t *)(smem + L.bc), *bk = (uint32_t *)(smem + L.bk), *bl = (uint32_t *)(smem + L.bl),
           *bp = (uint32_t *)(smem + L.bp), *bm = (uint32_t *)(smem + L.bm);
  uint32_t *ec = (uint32_t *)(smem + L.ec), *et = (uint32_t *)(smem + L.et);
  uint32_t *rs = (uint32_t *)(smem + L.rs), *re = (uint32_t *)(smem + L.re), *ri = (uint32_t *)(smem + L.ri);
  // ---- 1 decode: rounds of NT updates, one walk per update (register window over HBM);
  //      the round's counts are scanned and every lane writes its records in update order
  uint32_t NB = 0, NE = 0, NR = 0;
  uint32_t flags = 0; // 1 unsupported, 2 big DS table, 4 capacity, 8 huge block
  __syncthreads();
  for (uint32_t r0 = 0; r0 < U; r0 += NT) {
    const uint32_t i = r0 + t;
    uint32_t ubase = 0, ulen = 0, e = 0, shape = 0, w0f = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0, w5 = 0;
    uint32_t snb = 0, sne = 0, snr = 0;
    if (i < U) {
      const uint64_t a0 = b.upd_off[u0 + i], a1 = b.upd_off[u0 + i + 1];
      ubase = (uint32_t)(a0 - B0);
      ulen = (uint32_t)(a1 - a0);
      const uint2 *rp = (const uint2 *)(b.rec + (size_t)(u0 + i) * REC_WORDS);
      const uint2 x0 = rp[0], x1 = rp[1], x2 = rp[2];
      uint32_t w0 = x0.x;
      w1 = x0.y;
      w2 = x1.x;
      w3 = x1.y;
      w4 = x2.x;
      w5 = x2.y;
      if (STAMPS && (w0 & REC_SLOW)) atomicAdd((unsigned long long *)&o.stamps[(size_t)blockIdx.x * 16 + 12], 1ull);
      if (STAMPS && ((w0 >> 10) & 3) == REC_COMPLEX)
        atomicAdd((unsigned long long *)&o.stamps[(size_t)blockIdx.x * 16 + 13], 1ull);
      if (w0 & REC_SLOW) { // not a fast shape (or malformed): exact walk over HBM
        uint32_t w[6];
        walk_record_hbm(in + ubase, ulen, w);
        w0 = w[0];
        w1 = w[1];
        w2 = w[2];
        w3 = w[3];
        w4 = w[4];
        w5 = w[5];
      }
      w0f = w0;
      e = w0 & 0xFF;
      shape = (w0 >> 10) & 3;
      if (e) atomicMin(&misc[0], (i << 8) | e);
      if (w0 & REC_UNSUP) flags |= 1;
      if (w0 & REC_BIGDS) flags |= 2;
      if (w0 & REC_ORDER) flags |= 16;
      if (ulen >= (1u << 24)) flags |= 8;
      if (!e) {
        if (shape == REC_BLOCK) snb = 1;
        else if (shape == REC_DS) {
          sne = 1;
          snr = (w0 >> 12) & 3;
        } else if (shape == REC_COMPLEX) {
          snb = w1;
          sne = w2;
          snr = w3;
        }
      }
      // one update above a cap can never fit; clamping each lane to its cap also keeps the
      // 21-bit fields of the packed round scan below from wrapping (NT * cap < 2^21)
      if (snb > caps.b_cap || sne > caps.e_cap || snr > caps.r_cap) {
        flags |= 4;
        snb = sne = snr = 0;
      }
    }
    // packed scan: blocks | entries << 21 | ranges << 42 (each < 2^21 per round)
    uint64_t T;
    const uint64_t pk = (uint64_t)snb | ((uint64_t)sne << 21) | ((uint64_t)snr << 42);
    const uint64_t pre = bscan_sum64<NT>(pk, (uint64_t *)(misc + 2), T);
    const uint32_t pb = NB + (uint32_t)(pre & 0x1FFFFF), pe = NE + (uint32_t)((pre >> 21) & 0x1FFFFF),
                   pr = NR + (uint32_t)(pre >> 42);
    NB += (uint32_t)(T & 0x1FFFFF);
    NE += (uint32_t)((T >> 21) & 0x1FFFFF);
    NR += (uint32_t)(T >> 42);
    if (NB > caps.b_cap || NE > caps.e_cap || NR > caps.r_cap || __syncthreads_or(flags & 4)) {
      flags |= 4;
      break; // uniform: every lane sees the same totals / the same OR
    }
    if (i < U && !e) {
      if (shape == REC_BLOCK) {
        bc[pb] = w1;
        bk[pb] = w2;
        bl[pb] = w3;
        bp[pb] = ubase + w4;
        bm[pb] = w5;
      } else if (shape == REC_DS) {
        ec[pe] = w1;
        et[pe] = 0x80000000u | (i << 8);
        if (snr > 0) {
          rs[pr] = w2;
          re[pr] = w3;
          ri[pr] = pe;
        }
        if (snr > 1) {
          rs[pr + 1] = w4;
          re[pr + 1] = w5;
          ri[pr + 1] = pe;
        }
      } else if (w0f & REC_OVF) { // multi-record update decoded by k_decode
        if (STAMPS) atomicAdd((unsigned long long *)&o.stamps[(size_t)blockIdx.x * 16 + 15],
                              (unsigned long long)(5 * snb + 2 * sne + 3 * snr));
        const uint32_t *ov = b.ovf + w4;
        {
          for (uint32_t k = 0; k < snb; k++) {
            bc[pb + k] = ov[5 * k];
            bk[pb + k] = ov[5 * k + 1];
            bl[pb + k] = ov[5 * k + 2];
            bp[pb + k] = ubase + ov[5 * k + 3];
            bm[pb + k] = ov[5 * k + 4];
          }
          ov += 5 * snb;
          for (uint32_t k = 0; k < sne; k++) {
            ec[pe + k] = ov[k];
            et[pe + k] = ov[sne + k] | (i << 8); // table code from k_decode
          }
          ov += 2 * sne;
          for (uint32_t k = 0; k < snr; k++) {
            rs[pr + k] = ov[3 * k];
            re[pr + k] = ov[3 * k + 1];
            ri[pr + k] = pe + ov[3 * k + 2];
          }
        }
      } else if (shape == REC_COMPLEX && !(flags & 2)) {
        // not a one-record shape: walk the update again over HBM at its scanned positions
        if (STAMPS) atomicAdd((unsigned long long *)&o.stamps[(size_t)blockIdx.x * 16 + 14], 1ull);
        FastFill f{bc, bk, bl, bp, bm, ec, et, rs, re, ri, i, ubase, pb, pe, pr, 0};
        fill_hbm(in + ubase, ulen, &f);
      }
    }
  }
  if (flags) atomicOr(&misc[1], flags);
  __syncthreads();
  YM_STAMP(1);
  {
    const uint32_t ek = misc[0], fl = misc[1];
    if (ek == 0xFFFFFFFFu && (fl & 30)) { // capacity: tiled kernel; big DS table, huge block,
      handover((fl & 4) && !(fl & 16) ? 2 : 1); // client sections out of order: exact engine
      return;
    }
    if (ek != 0xFFFFFFFFu || fl) {
      if (t == 0) {
        o.status[d] = (uint8_t)(ek != 0xFFFFFFFFu ? (ek & 0xFF) : E_UNSUPPORTED);
        o.path[d] = 0;
        o.out_len[d] = 0;
        o.out_start[d] = slot;
      }
      return;
    }
  }
  YM_STAMP(2);
  // ---- 3 sort blocks by (client desc, clock asc, input order).
  // Stable counting sort by client rank (<= 32 distinct clients: LDS table), then a
  // per-client clock-order check; LDS bitonic only when that check fails.
  uint64_t *skey = (uint64_t *)(smem + L.skey);
  uint32_t *sval = (uint32_t *)(smem + L.sval);
  {
    uint64_t *btab = (uint64_t *)(misc + 256); // [BTAB] (client << 32 | rank), ~0 = empty
    for (uint32_t i = t; i < BTAB; i += NT) btab[i] = ~0ull;
    if (t == 0) sc[3] = 0;
    __syncthreads();
    const uint32_t per0 = (NB + NT - 1) / NT, k0 = t * per0, k1 = k0 + per0 < NB ? k0 + per0 : NB;
    uint32_t overflow = 0;
    for (uint32_t k = k0; k < k1; k++) {
      uint32_t c = bc[k];
      if (k > k0 && bc[k - 1] == c) continue;
      uint32_t h = mix32(c) >> 26; // 64 slots
      for (uint32_t probe = 0;; probe++) {
        if (probe == BTAB) {
          overflow = 1;
          break;
        }
        uint64_t cur = btab[h];
        if (cur == ~0ull) {
          uint64_t prev = atomicCAS((unsigned long long *)&btab[h], ~0ull, ((uint64_t)c << 32));
          if (prev == ~0ull) {
            atomicAdd(&sc[3], 1u);
            break;
          }
          cur = prev;
        }
        if ((uint32_t)(cur >> 32) == c) break;
        h = (h + 1) & (BTAB - 1);
      }
    }
    overflow = __syncthreads_or(overflow);
    const uint32_t ncl = sc[3];
    bool counting = !overflow && ncl <= 8 && NB <= 65535;
    if (counting) {
      // rank = number of distinct clients greater than this one (lane per table slot)
      uint64_t mine = t < BTAB ? btab[t] : ~0ull;
      uint32_t r = 0;
      if (mine != ~0ull)
        for (uint32_t j = 0; j < BTAB; j++) {
          uint64_t o2 = btab[j];
          r += (o2 != ~0ull && (uint32_t)(o2 >> 32) > (uint32_t)(mine >> 32));
        }
      __syncthreads();
      if (mine != ~0ull) btab[t] = (mine & 0xFFFFFFFF00000000ull) | r;
      __syncthreads();
      auto rank_of = [&](uint32_t c) -> uint32_t {
        uint32_t h = mix32(c) >> 26;
        while ((uint32_t)(btab[h] >> 32) != c) h = (h + 1) & (BTAB - 1);
        return (uint32_t)btab[h];
      };
      // Two packed 64-bit scans (ranks 0-3, 4-7; 16-bit counters, NB <= 65535), kept in
      // registers: P0/P1 field r = next sorted position of this lane's rank-r blocks.
      uint64_t P0 = 0, P1 = 0;
      for (uint32_t k = k0; k < k1; k++) {
        uint32_t r = rank_of(bc[k]);
        uint64_t inc = 1ull << (16 * (r & 3));
        if (r < 4) P0 += inc;
        else P1 += inc;
      }
      uint64_t T0, T1;
      P0 = bscan_sum64<NT>(P0, (uint64_t *)(misc + 2), T0);
      P1 = bscan_sum64<NT>(P1, (uint64_t *)(misc + 2), T1);
      {
        // add rank starts (exclusive sum of rank totals) into every field
        uint64_t S0 = 0, S1 = 0;
        uint32_t start = 0;
#pragma unroll
        for (uint32_t r = 0; r < 8; r++) {
          uint64_t T = r < 4 ? T0 : T1;
          uint32_t tot = (uint32_t)((T >> (16 * (r & 3))) & 0xFFFF);
          if (r < 4) S0 |= (uint64_t)start << (16 * r);
          else S1 |= (uint64_t)start << (16 * (r - 4));
          start += tot;
        }
        P0 += S0;
        P1 += S1;
      }
      for (uint32_t k = k0; k < k1; k++) {
        uint32_t r = rank_of(bc[k]);
        uint32_t sh = 16 * (r & 3);
        uint32_t pos;
        if (r < 4) {
          pos = (uint32_t)((P0 >> sh) & 0xFFFF);
          P0 += 1ull << sh;
        } else {
          pos = (uint32_t)((P1 >> sh) & 0xFFFF);
          P1 += 1ull << sh;
        }
        sval[pos] = k;
        skey[pos] = ((uint64_t)(~bc[k]) << 32) | bk[k];
      }
      __syncthreads();
      // clock order within each client run
      uint32_t bad = 0;
      for (uint32_t j = t; j + 1 < NB; j += NT)
        if (skey[j] > skey[j + 1]) bad = 1;
      counting = !__syncthreads_or(bad);
    }
    if (!counting) {
      uint32_t n2 = pow2ceil(NB);
      for (uint32_t j = t; j < n2; j += NT) {
        skey[j] = j < NB ? (((uint64_t)(~bc[j]) << 32) | bk[j]) : ~0ull;
        sval[j] = j;
      }
      __syncthreads();
      bitonic<NT>(skey, sval, n2);
    }
  }
  YM_STAMP(3);
  // ---- 4 register chunk: lane t owns sorted positions j = t*PER + k (k < PER); the
  //      records are read once through sval into registers for classify, sizes, write
  const uint32_t j0 = t * PER;
  uint32_t rc[PER], rk[PER], rl[PER], rp[PER], rm[PER], rE[PER], rF[PER], rS[PER];
  bool hd[PER];
  {
    bool havepc = false;
    uint32_t pc = 0;
    if (j0 > 0 && j0 < NB) {
      pc = bc[sval[j0 - 1]];
      havepc = true;
    }
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t j = j0 + k;
      rc[k] = rk[k] = rl[k] = rp[k] = rm[k] = rE[k] = rF[k] = rS[k] = 0;
      hd[k] = false;
      if (j < NB) {
        const uint32_t r = sval[j];
        rc[k] = bc[r];
        rk[k] = bk[r];
        rl[k] = bl[r];
        rp[k] = bp[r];
        rm[k] = bm[r];
      }
    }
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t j = j0 + k;
      if (k == 0) hd[0] = j < NB && (j == 0 || !havepc || pc != rc[0]);
      else hd[k] = j < NB && rc[k] != rc[k - 1];
    }
  }
  // classify: segmented exclusive max of block ends (segments = clients)
  {
    uint32_t lf = 0, lv = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (j0 + k >= NB) continue;
      const uint32_t e = rk[k] + rl[k];
      if (hd[k]) {
        lf = 1;
        lv = e;
      } else {
        lv = OpMax::f(lv, e);
      }
    }
    uint32_t pf, pv;
    bscan_seg<NT, OpMax>(lf, lv, ws, pf, pv);
    uint32_t run = pv, viol = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (j0 + k >= NB) continue;
      const uint32_t e = rk[k] + rl[k];
      const uint32_t E = hd[k] ? 0 : run;
      uint32_t flag = 0;
      if (rl[k] == 0) viol |= 2; // zero-length GC: leave to the exact engine
      if (hd[k] || rk[k] >= E) {
        flag = 1;                               // keep
        if (!hd[k] && rk[k] > E) flag |= 2;     // Skip of (k - E) before it
      } else if (e > E) {
        viol |= 1; // partial overlap: the tiled kernel's overlap mode
      }
      rE[k] = E;
      rF[k] = flag;
      run = hd[k] ? e : OpMax::f(run, e);
    }
    const uint32_t vz = __syncthreads_or(viol & 2);
    if (vz || __syncthreads_or(viol & 1)) {
      handover(vz ? 1 : 2);
      return;
    }
  }
  // dropped blocks must be covered with a later start, or byte-identical to the last kept block
  {
    uint32_t lf = 0, lv = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (j0 + k >= NB) continue;
      if (hd[k]) {
        lf = 1;
        lv = 0;
      }
      if (rF[k] & 1) lv = j0 + k + 1;
    }
    uint32_t pf, pv;
    bscan_seg<NT, OpMax>(lf, lv, ws, pf, pv);
    uint32_t last = pv, viol = 0, pan = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (j0 + k >= NB) continue;
      if (hd[k]) last = 0;
      if (!(rF[k] & 1)) {
        const uint32_t kr = sval[last - 1];
        if (bk[kr] == rk[k]) { // same start: must be an exact duplicate (kind, length, bytes)
          const uint32_t la = bm[kr] >> 8, lb = rm[k] >> 8;
          bool same = la == lb && (bm[kr] & 3) == (rm[k] & 3) && bl[kr] == rl[k];
          if (same) same = equal_window(in + bp[kr], in + rp[k], la);
          if (!same) viol = 1;
        }
      } else {
        last = j0 + k + 1;
        if (rm[k] & 8) pan = 1; // yrs panics encoding a kept String that is not valid UTF-8
      }
    }
    const uint32_t vp = (__syncthreads_or(viol) ? 1u : 0u) | (__syncthreads_or(pan) ? 2u : 0u); // (0/1 each)
    if (vp & 1) { // same-clock blocks that differ: the tiled kernel's overlap mode
      handover(2);
      return;
    }
    if (vp & 2) {
      if (t == 0) {
        o.path[d] = 0;
        o.status[d] = E_PANIC;
        o.out_len[d] = 0;
        o.out_start[d] = slot;
      }
      return;
    }
  }
  YM_STAMP(4);
  // ---- 6a block section sizes: per client header + (Skip) + canonical block bytes
  uint32_t blocks_size, NC;
  uint32_t *sseg = (uint32_t *)(smem + L.skey); // blocks emitted per client (skey is free now)
  {
    uint32_t nh = 0, lf = 0, lv = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (j0 + k >= NB) continue;
      const uint32_t c = (rF[k] & 1) + ((rF[k] >> 1) & 1);
      if (hd[k]) {
        nh++;
        lf = 1;
        lv = c;
      } else {
        lv += c;
      }
    }
    const uint32_t hpre = bscan_sum<NT>(nh, ws, NC);
    uint32_t pf, pv;
    bscan_seg<NT, OpSum>(lf, lv, ws, pf, pv);
    // tail of the chunk's last element: head of the next sorted position
    const uint32_t jl = j0 + PER;
    const bool next_head = jl >= NB || (jl < NB && bc[sval[jl]] != rc[PER - 1]);
    uint32_t rank = hpre, run = pv;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (j0 + k >= NB) continue;
      const uint32_t c = (rF[k] & 1) + ((rF[k] >> 1) & 1);
      if (hd[k]) {
        rank++;
        run = c;
      } else {
        run += c;
      }
      const bool tail = k + 1 < PER ? (j0 + k + 1 >= NB || hd[k + 1]) : next_head;
      if (tail) sseg[rank - 1] = run;
    }
    __syncthreads();
    uint32_t ls = 0;
    rank = hpre;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (j0 + k >= NB) continue;
      uint32_t s = 0;
      if (hd[k]) {
        rank++;
        const uint32_t cnt = sseg[rank - 1];
        rF[k] |= cnt << 8;
        s += varlen(cnt) + varlen(rc[k]) + varlen(rk[k]);
      }
      if (rF[k] & 2) s += 1 + varlen(rk[k] - rE[k]);
      if (rF[k] & 1) s += canon_size(in, nbytes, rp[k], rc[k], rk[k], rl[k], rm[k]);
      rS[k] = s;
      ls += s;
    }
    uint32_t tot;
    const uint32_t pre = bscan_sum<NT>(ls, ws, tot);
    const uint32_t base = varlen(NC);
    uint32_t pos = base + pre;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t s = rS[k];
      rS[k] = pos;
      pos += s;
    }
    blocks_size = base + tot;
  }
  YM_STAMP(5);
  // ---- 6b write the block section into the document's slot
  uint8_t *out = o.out + slot;
  // Lanes write their pieces into LDS at the destination's 16-byte phase, then the
  // workgroup stores whole aligned 16-byte chunks (partial end chunks byte by byte: the
  // neighbouring bytes belong to other slots).  Sections larger than the stage are written
  // straight to HBM.
  const uint32_t phase = (uint32_t)((uintptr_t)out & 15);
  const bool staged = phase + blocks_size <= L.total - L.stage;
  uint8_t *wdst = staged ? smem + L.stage + phase : out;
  if (blocks_size <= cap) {
    if (t == 0) {
      Writer w{wdst, 0};
      w_var(w, NC);
    }
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (j0 + k >= NB) continue;
      Writer w{wdst, rS[k]};
      if (hd[k]) {
        w_var(w, rF[k] >> 8);
        w_var(w, rc[k]);
        w_var(w, rk[k]);
      }
      if (rF[k] & 2) {
        w.u8(10);
        w_var(w, rk[k] - rE[k]);
      }
      if (rF[k] & 1) {
        if ((rm[k] & 4) && !(rm[k] & 8)) {
          Writer w2 = w; // only the out-of-line re-encode takes a Writer by reference
          emit_block(in, nbytes, rp[k], rc[k], rk[k], rl[k], 0, w2);
        } else {
          copy_bytes16(w.p + w.n, in + rp[k], rm[k] >> 8);
        }
      }
    }
    if (staged) {
      __syncthreads();
      const uint8_t *st = smem + L.stage;
      uint8_t *gbase = out - phase;
      const uint32_t span = phase + blocks_size, nch = (span + 15) >> 4;
      for (uint32_t c = t; c < nch; c += NT) {
        const uint32_t b0 = c << 4, lo = b0 < phase ? phase : b0, hi = b0 + 16 < span ? b0 + 16 : span;
        if (lo == b0 && hi == b0 + 16) {
          *(uint4 *)(gbase + b0) = *(const uint4 *)(st + b0);
        } else {
          for (uint32_t q = lo; q < hi; q++) gbase[q] = st[q];
        }
      }
    }
  }
  __syncthreads();

  YM_STAMP(6);
  // ---- 5 DeleteSet: distinct clients in yrs' table order, union of ranges
  uint64_t *dkey = (uint64_t *)(smem + L.dkey);
  uint32_t *dval = (uint32_t *)(smem + L.dval);
  const uint32_t RSZ = pow2ceil(caps.r_cap > caps.e_cap ? caps.r_cap : caps.e_cap);
  uint32_t *d_client = (uint32_t *)(smem + L.dcl), *d_first = (uint32_t *)(smem + L.dfirst),
           *d_aux = (uint32_t *)(smem + L.dord);
  // 5a distinct clients of live entries and their first occurrence (upd << 8 | tpos):
  //    LDS open-addressing table, 64-bit CAS insert, atomicMin on a hit
  uint64_t *dtab = (uint64_t *)(smem + L.dtab);
  const uint32_t TS = DTAB_SLOTS;
  for (uint32_t j = t; j < TS; j += NT) dtab[j] = ~0ull;
  __syncthreads();
  uint32_t tovf = 0;
  for (uint32_t j = t; j < NE && !tovf; j += NT) {
    if (!(et[j] & 0x80000000u)) continue;
    const uint32_t c = ec[j];
    const uint64_t v = ((uint64_t)c << 32) | (et[j] & 0x7FFFFFFFu);
    uint32_t h = mix32(c) & (TS - 1);
    for (;;) {
      uint64_t cur = dtab[h];
      if (cur == ~0ull) {
        cur = atomicCAS((unsigned long long *)&dtab[h], ~0ull, (unsigned long long)v);
        if (cur == ~0ull) break;
      }
      if ((uint32_t)(cur >> 32) == c) {
        atomicMin((unsigned long long *)&dtab[h], (unsigned long long)v);
        break;
      }
      h = (h + 1) & (TS - 1);
      if (h == (mix32(c) & (TS - 1))) { // table full: more distinct clients than the fast path keeps
        tovf = 1;
        break;
      }
    }
  }
  if (__syncthreads_or(tovf)) {
    handover(2);
    return;
  }
  // compact the occupied slots, then order them by client (rank sort: D is small)
  uint32_t D;
  {
    const uint32_t pt = TS / NT ? TS / NT : 1, s0 = t * pt, s1 = s0 + pt < TS ? s0 + pt : TS;
    uint32_t nh = 0;
    for (uint32_t j = s0; j < s1; j++) nh += dtab[j] != ~0ull;
    uint32_t pre = bscan_sum<NT>(nh, ws, D);
    for (uint32_t j = s0; j < s1; j++)
      if (dtab[j] != ~0ull && pre < DCAP) dkey[pre++] = dtab[j];
  }
  if (D > DCAP) {
    handover(2);
    return;
  }
  __syncthreads();
  for (uint32_t j = t; j < D; j += NT) {
    const uint64_t kj = dkey[j];
    uint32_t r = 0;
    for (uint32_t q = 0; q < D; q++) r += dkey[q] < kj; // clients are distinct
    d_client[r] = (uint32_t)(kj >> 32);
    d_first[r] = (uint32_t)kj;
  }
  __syncthreads();
  YM_STAMP(7);
  // 5b yrs' table order (IdSet::merge inserts in first-occurrence order, hashbrown layout)
  if (t == 0) {
    // insertion order: sort ranks by first occurrence (insertion sort; D is small in practice)
    uint32_t *ord = d_aux;
    for (uint32_t i = 0; i < D; i++) {
      uint32_t x = i, j = i;
      while (j > 0 && d_first[ord[j - 1]] > d_first[x]) {
        ord[j] = ord[j - 1];
        j--;
      }
      ord[j] = x;
    }
    // emulate the table: slots hold rank+1; reuse dkey (as u32) for slots — dkey is free now
    uint32_t *slot_arr = (uint32_t *)dkey;
    uint32_t slot_cap = 2 * RSZ; // u32 capacity of dkey region
    uint32_t buckets = 0, items = 0, growth = 0;
    auto ctrl_empty = [&](uint32_t idx) -> bool {
      if (idx < buckets) return slot_arr[idx] == 0;
      if (buckets < 16) return idx < 16 ? true : slot_arr[idx - 16] == 0;
      return slot_arr[idx - buckets] == 0;
    };
    auto find_slot = [&](uint32_t key) -> uint32_t {
      uint32_t mask = buckets - 1, pos = key & mask, stride = 0;
      for (;;) {
        for (uint32_t j = 0; j < 16; j++) {
          if (ctrl_empty(pos + j)) {
            uint32_t index = (pos + j) & mask;
            if (slot_arr[index] != 0)
              for (uint32_t k = 0; k < buckets; k++)
                if (slot_arr[k] == 0) return k;
            return index;
          }
        }
        stride += 16;
        pos = (pos + stride) & mask;
      }
    };
    uint32_t ok = 1;
    uint32_t *tmp = dval; // resize scratch
    for (uint32_t i = 0; i < D && ok; i++) {
      if (growth == 0) {
        uint64_t full = buckets ? mask_to_cap(buckets - 1) : 0;
        uint64_t need = items + 1;
        uint64_t nb = cap_to_buckets(need > full + 1 ? need : full + 1);
        if (nb > slot_cap / 2) {
          ok = 0;
          break;
        }
        uint32_t ob = buckets;
        for (uint32_t q = 0; q < ob; q++) tmp[q] = slot_arr[q];
        buckets = (uint32_t)nb;
        for (uint32_t q = 0; q < buckets; q++) slot_arr[q] = 0;
        for (uint32_t q = 0; q < ob; q++)
          if (tmp[q]) slot_arr[find_slot(d_client[tmp[q] - 1])] = tmp[q];
        growth = (uint32_t)mask_to_cap(buckets - 1) - items;
      }
      uint32_t rk = ord[i];
      slot_arr[find_slot(d_client[rk])] = rk + 1;
      items++;
      growth--;
    }
    // iteration order -> ord (rank list)
    uint32_t k = 0;
    for (uint32_t q = 0; q < buckets && ok; q++)
      if (slot_arr[q]) ord[k++] = slot_arr[q] - 1;
    sc[1] = ok;
  }
  __syncthreads();
  if (!sc[1]) {
    handover(2);
    return;
  }
  YM_STAMP(8);
  // 5c' DeleteSet union by bitmap.  When every live range is non-empty and the clients'
  //     clock windows [min start, max end) fit BMAP_WORDS words, each range sets its bits
  //     in its client's window and the union's components are the runs of set bits:
  //     ranges join when they overlap or touch (IdRange::squash, id_set.rs:129-164), the
  //     runs come out in start order, so no range sort is needed.  (An empty range [c, c)
  //     is a component of its own in yrs when isolated: the sort path below keeps that.)
  {
    uint32_t *cmin = d_first;                      // first occurrences are no longer needed
    uint32_t *cmax = misc + 128;                   // [DCAP] (misc words 128..191 are free here)
    uint32_t *woff = (uint32_t *)(smem + L.dbeg);  // [D + 1] word offset of each client's window
    uint32_t *bmp = (uint32_t *)(smem + L.dkey);   // [BMAP_WORDS]
    uint32_t *cb = bmp + BMAP_WORDS;               // [BMAP_WORDS + 1] components before each word
    uint32_t *cst = (uint32_t *)(smem + L.coff);   // [NR] component start
    uint32_t *cen = (uint32_t *)(smem + L.chead);  // [NR] component end
    uint32_t *cof = (uint32_t *)(smem + L.dtab);   // [NR + 1] component byte offsets
    auto rank_of = [&](uint32_t c) -> uint32_t {
      uint32_t lo = 0, hi = D;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (d_client[mid] < c) lo = mid + 1;
        else hi = mid;
      }
      return lo;
    };
    for (uint32_t r = t; r < D; r += NT) {
      cmin[r] = 0xFFFFFFFFu;
      cmax[r] = 0;
    }
    __syncthreads();
    uint32_t bad = 0;
    for (uint32_t j = t; j < NR; j += NT) {
      if (!(et[ri[j]] & 0x80000000u)) continue;
      if (re[j] == rs[j]) {
        bad = 1;
        continue;
      }
      const uint32_t r = rank_of(ec[ri[j]]);
      atomicMin(&cmin[r], rs[j]);
      atomicMax(&cmax[r], re[j]);
    }
    bad = __syncthreads_or(bad);
    if (!bad && t == 0) {
      uint32_t w = 0;
      for (uint32_t r = 0; r < D; r++) {
        woff[r] = w;
        if (cmax[r] > cmin[r]) {
          const uint64_t span = ((uint64_t)cmax[r] - cmin[r] + 31) >> 5;
          w = span > BMAP_WORDS ? BMAP_WORDS + 1 : w + (uint32_t)span;
          if (w > BMAP_WORDS) w = BMAP_WORDS + 1;
        }
      }
      woff[D] = w;
      sc[3] = w;
    }
    __syncthreads();
    const uint32_t W = bad ? BMAP_WORDS + 1 : sc[3];
    if (W <= BMAP_WORDS) {
      for (uint32_t k = t; k < W; k += NT) bmp[k] = 0;
      __syncthreads();
      for (uint32_t j = t; j < NR; j += NT) {
        if (!(et[ri[j]] & 0x80000000u)) continue;
        const uint32_t r = rank_of(ec[ri[j]]);
        uint32_t a = rs[j] - cmin[r];
        const uint32_t z = re[j] - cmin[r];
        while (a < z) {
          const uint32_t wi = a >> 5, bo = a & 31, nb = (z - a < 32 - bo) ? z - a : 32 - bo;
          const uint32_t mask = (nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1)) << bo;
          atomicOr(&bmp[woff[r] + wi], mask);
          a += nb;
        }
      }
      __syncthreads();
      YM_STAMP(9);
      // runs: starts / ends per word, components before each word (block scan)
      const uint32_t wpl = (W + NT - 1) / NT, k0 = t * wpl, k1 = k0 + wpl < W ? k0 + wpl : W;
      uint32_t nst = 0;
      for (uint32_t k = k0; k < k1; k++) {
        const uint32_t r = [&]() {
          uint32_t lo = 0, hi = D;
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (woff[mid + 1] <= k) lo = mid + 1;
            else hi = mid;
          }
          return lo;
        }();
        const uint32_t bits = bmp[k], prev = k > woff[r] ? bmp[k - 1] >> 31 : 0;
        nst += __popc(bits & ~((bits << 1) | prev));
      }
      uint32_t NCD;
      uint32_t pre = bscan_sum<NT>(nst, ws, NCD);
      for (uint32_t k = k0; k < k1; k++) {
        uint32_t lo = 0, hi = D;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (woff[mid + 1] <= k) lo = mid + 1;
          else hi = mid;
        }
        const uint32_t r = lo;
        const uint32_t bits = bmp[k], prev = k > woff[r] ? bmp[k - 1] >> 31 : 0;
        const uint32_t next = k + 1 < woff[r + 1] ? bmp[k + 1] & 1 : 0;
        uint32_t st = bits & ~((bits << 1) | prev), en = bits & ~((bits >> 1) | (next << 31));
        const uint32_t st0 = st, base = cmin[r] + 32 * (k - woff[r]);
        cb[k] = pre;
        while (st) {
          const uint32_t q = __builtin_ctz(st);
          cst[pre + __popc(st0 & ((1u << q) - 1))] = base + q;
          st &= st - 1;
        }
        while (en) {
          const uint32_t q = __builtin_ctz(en);
          const uint32_t upto = q == 31 ? st0 : (st0 & ((2u << q) - 1));
          cen[pre + __popc(upto) - 1] = base + q + 1;
          en &= en - 1;
        }
        pre += __popc(st0);
      }
      if (t == 0) cb[W] = NCD;
      __syncthreads();
      // component byte sizes -> offsets
      const uint32_t cpl = (NCD + NT - 1) / NT, c0 = t * cpl, c1 = c0 + cpl < NCD ? c0 + cpl : NCD;
      uint32_t ls = 0;
      for (uint32_t c = c0; c < c1; c++) ls += varlen(cst[c]) + varlen(cen[c] - cst[c]);
      uint32_t TS;
      uint32_t po = bscan_sum<NT>(ls, ws, TS);
      for (uint32_t c = c0; c < c1; c++) {
        cof[c] = po;
        po += varlen(cst[c]) + varlen(cen[c] - cst[c]);
      }
      if (t == 0) cof[NCD] = TS;
      __syncthreads();
      YM_STAMP(10);
      uint32_t *r_ncomp = (uint32_t *)(smem + L.dnc), *r_off = (uint32_t *)(smem + L.doff);
      if (t == 0) { // client headers in yrs' iteration order (d_aux)
        uint32_t pos = varlen(D);
        for (uint32_t i = 0; i < D; i++) {
          const uint32_t r = d_aux[i];
          const uint32_t ca = cb[woff[r]], cz = cb[woff[r + 1]];
          r_ncomp[r] = cz - ca;
          r_off[r] = pos;
          pos += varlen(d_client[r]) + varlen(cz - ca) + (cof[cz] - cof[ca]);
        }
        sc[2] = pos;
      }
      __syncthreads();
      const uint64_t total = (uint64_t)blocks_size + sc[2];
      if (total > cap) {
        handover();
        return;
      }
      uint8_t *dso = out + blocks_size;
      if (t == 0) {
        Writer w{dso, 0};
        w_var(w, D);
      }
      for (uint32_t r = t; r < D; r += NT) {
        Writer w{dso, r_off[r]};
        w_var(w, d_client[r]);
        w_var(w, r_ncomp[r]);
      }
      for (uint32_t c = t; c < NCD; c += NT) {
        uint32_t lo = 0, hi = D; // client of component c: last r with cb[woff[r]] <= c
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (cb[woff[mid + 1]] <= c) lo = mid + 1;
          else hi = mid;
        }
        const uint32_t r = lo;
        Writer w{dso, r_off[r] + varlen(d_client[r]) + varlen(r_ncomp[r]) + (cof[c] - cof[cb[woff[r]]])};
        w_var(w, cst[c]);
        w_var(w, cen[c] - cst[c]);
      }
      if (t == 0) {
        o.path[d] = 0;
        o.status[d] = 0;
        o.out_len[d] = total;
        o.out_start[d] = slot;
      }
      YM_STAMP(11);
      return;
    }
  }
  // 5c ranges of live entries sorted by (client, start, index): rank sort, every lane
  //    counts the smaller keys with LDS broadcast reads (no barrier stages)
  {
    uint64_t *tkey = dtab; // >= NR slots
    uint32_t unsorted = 0;
    for (uint32_t j = t; j < NR; j += NT) {
      bool live = et[ri[j]] & 0x80000000u;
      tkey[j] = live ? (((uint64_t)ec[ri[j]] << 32) | rs[j]) : ~0ull;
    }
    __syncthreads();
    for (uint32_t j = t; j + 1 < NR; j += NT)
      if (tkey[j] > tkey[j + 1]) unsorted = 1;
    unsorted = __syncthreads_or(unsorted);
    if (unsorted) {
      // bottom-up stable merge sort, one barrier per level: an element of a left run lands
      // at base + i + #(right-run keys < k), of a right run at base + i + #(left-run keys
      // <= k) (binary searches).  Equal keys keep index order, exactly like a rank sort by
      // (key, index).  cmp_end is free until 5d and carries the indices of the tkey side.
      uint64_t *ka = tkey, *kb = dkey;
      uint32_t *ia = (uint32_t *)(smem + L.cend), *ib = dval;
      // levels w < 64 in registers: each wave bitonic-sorts 64-element segments by
      // (key, index) with lane shuffles (index makes keys distinct, so this equals the
      // stable order); padding lanes carry (~0, index >= NR) and sort last
      {
        const uint32_t lane = t & 63;
        for (uint32_t jb = t - lane; jb < NR; jb += NT) { // uniform per wave
          const uint32_t j = jb + lane;
          uint64_t key = j < NR ? tkey[j] : ~0ull;
          uint32_t idx = j;
#pragma unroll
          for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
            for (uint32_t sft = k >> 1; sft > 0; sft >>= 1) {
              const uint32_t okl = __shfl_xor((uint32_t)key, (int)sft, 64);
              const uint32_t okh = __shfl_xor((uint32_t)(key >> 32), (int)sft, 64);
              const uint32_t oi = __shfl_xor(idx, (int)sft, 64);
              const uint64_t ok = ((uint64_t)okh << 32) | okl;
              const bool other_less = ok < key || (ok == key && oi < idx);
              const bool up = (lane & k) == 0, lower = (lane & sft) == 0;
              if (lower == up ? other_less : !other_less) {
                key = ok;
                idx = oi;
              }
            }
          }
          if (j < NR) {
            kb[j] = key;
            ib[j] = idx;
          }
        }
      }
      __syncthreads();
      {
        uint64_t *tk = ka; ka = kb; kb = tk;
        uint32_t *ti = ia; ia = ib; ib = ti;
      }
      for (uint32_t w = 64; w < NR; w <<= 1) {
        for (uint32_t j = t; j < NR; j += NT) {
          const uint64_t kj = ka[j];
          const uint32_t run = j / w, i = j - run * w;
          const bool left = !(run & 1);
          const uint32_t base = (left ? run : run - 1) * w;
          uint32_t lo = left ? base + w : base, hi = left ? base + 2 * w : base + w;
          if (lo > NR) lo = NR;
          if (hi > NR) hi = NR;
          const uint32_t b0 = lo;
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint64_t km = ka[mid];
            if (left ? (km < kj) : (km <= kj)) lo = mid + 1;
            else hi = mid;
          }
          const uint32_t dst = base + i + (lo - b0);
          kb[dst] = kj;
          ib[dst] = ia[j];
        }
        __syncthreads();
        uint64_t *tk = ka; ka = kb; kb = tk;
        uint32_t *ti = ia; ia = ib; ib = ti;
      }
      if (ka != dkey)
        for (uint32_t j = t; j < NR; j += NT) {
          dkey[j] = ka[j];
          dval[j] = ia[j];
        }
    } else {
      for (uint32_t j = t; j < NR; j += NT) {
        dkey[j] = tkey[j];
        dval[j] = j;
      }
    }
    __syncthreads();
  }
  // live count
  uint32_t NL;
  {
    uint32_t c = 0;
    for (uint32_t j = t; j < NR; j += NT) c += dkey[j] != ~0ull;
    bscan_sum<NT>(c, ws, NL);
  }
  YM_STAMP(9);
  // 5d segmented union over sorted live ranges: comp heads, comp end, comp size at comp tails
  uint32_t *cmp_end = (uint32_t *)(smem + L.cend);
  uint32_t *cmp_off = (uint32_t *)(smem + L.coff);
  uint32_t *cmp_head = (uint32_t *)(smem + L.chead);
  const uint32_t pr = (NL + NT - 1) / NT, r0 = t * pr, r1 = r0 + pr < NL ? r0 + pr : NL;
  {
    uint32_t lf = 0, lv = 0;
    for (uint32_t j = r0; j < r1; j++) {
      bool chead = j == 0 || (dkey[j] >> 32) != (dkey[j - 1] >> 32);
      uint32_t e = re[dval[j]];
      if (chead) {
        lf = 1;
        lv = e;
      } else
        lv = OpMax::f(lv, e);
    }
    uint32_t pf, pv;
    bscan_seg<NT, OpMax>(lf, lv, ws, pf, pv);
    uint32_t run = pv;
    for (uint32_t j = r0; j < r1; j++) {
      bool chead = j == 0 || (dkey[j] >> 32) != (dkey[j - 1] >> 32);
      uint32_t s0 = (uint32_t)dkey[j], e = re[dval[j]];
      uint32_t h = chead ? 3u : (s0 > run ? 1u : 0u); // bit0 component head, bit1 client head
      cmp_head[j] = h;
      run = chead ? e : OpMax::f(run, e);
      cmp_end[j] = run; // inclusive running max within client
    }
  }
  __syncthreads();
  // component start propagated to its tail; component size at tails
  uint32_t ds_comp_total;
  {
    uint32_t lf = 0, lv = 0;
    for (uint32_t j = r0; j < r1; j++) {
      if (cmp_head[j] & 1) {
        lf = 1;
        lv = (uint32_t)dkey[j];
      }
    }
    uint32_t pf, pv;
    bscan_seg<NT, OpFirst>(lf, lv, ws, pf, pv);
    uint32_t cs = pv;
    uint32_t ls = 0;
    for (uint32_t j = r0; j < r1; j++) {
      if (cmp_head[j] & 1) cs = (uint32_t)dkey[j];
      bool tail = j + 1 == NL || (cmp_head[j + 1] & 1);
      uint32_t s = tail ? varlen(cs) + varlen(cmp_end[j] - cs) : 0;
      ls += s;
    }
    uint32_t pre = bscan_sum<NT>(ls, ws, ds_comp_total);
    // offsets of component bytes within the concatenation (client order = sorted order)
    cs = pv;
    uint32_t pos = pre;
    for (uint32_t j = r0; j < r1; j++) {
      if (cmp_head[j] & 1) cs = (uint32_t)dkey[j];
      bool tail = j + 1 == NL || (cmp_head[j + 1] & 1);
      uint32_t s = tail ? varlen(cs) + varlen(cmp_end[j] - cs) : 0;
      cmp_off[j] = pos;
      pos += s;
      // stash component start for the writer in the key's low half (no longer needed as key)
      if (tail) dkey[j] = (dkey[j] & 0xFFFFFFFF00000000ull) | cs;
    }
    if (t == 0) cmp_off[NL] = ds_comp_total;
  }
  __syncthreads();
  YM_STAMP(10);
  // 5e per distinct client (rank r, ascending client): range segment, #components, bytes
  // d_aux[0..D) holds iteration order; compute per-rank [rb, re) by binary search
  uint32_t *r_beg = (uint32_t *)(smem + L.dbeg);
  uint32_t *r_ncomp = (uint32_t *)(smem + L.dnc);
  uint32_t *r_off = (uint32_t *)(smem + L.doff);
  for (uint32_t r = t; r < D; r += NT) {
    uint32_t c = d_client[r];
    uint32_t lo = 0, hi = NL;
    while (lo < hi) {
      uint32_t mid = (lo + hi) / 2;
      if ((uint32_t)(dkey[mid] >> 32) < c) lo = mid + 1;
      else hi = mid;
    }
    uint32_t a = lo;
    hi = NL;
    while (lo < hi) {
      uint32_t mid = (lo + hi) / 2;
      if ((uint32_t)(dkey[mid] >> 32) <= c) lo = mid + 1;
      else hi = mid;
    }
    uint32_t bnd = lo, nc = 0;
    for (uint32_t j = a; j < bnd; j++) nc += cmp_head[j] & 1;
    r_beg[r] = a;
    r_ncomp[r] = nc;
    r_off[r] = bnd; // end, temporarily
  }
  __syncthreads();
  // client byte sizes in iteration order -> offsets (single lane; D is small)
  if (t == 0) {
    uint32_t pos = varlen(D);
    for (uint32_t i = 0; i < D; i++) {
      uint32_t r = d_aux[i];
      uint32_t a = r_beg[r], bnd = r_off[r];
      uint32_t bytes = cmp_off[bnd] - cmp_off[a];
      uint32_t hdr = varlen(d_client[r]) + varlen(r_ncomp[r]);
      r_off[r] = pos; // header position of client r
      pos += hdr + bytes;
    }
    sc[2] = pos;
  }
  __syncthreads();
  const uint32_t ds_size = sc[2];
  const uint64_t total = (uint64_t)blocks_size + ds_size;
  if (total > cap) {
    handover();
    return;
  }
  uint8_t *dso = out + blocks_size;
  if (t == 0) {
    Writer w{dso, 0};
    w_var(w, D);
  }
  for (uint32_t r = t; r < D; r += NT) {
    Writer w{dso, r_off[r]};
    w_var(w, d_client[r]);
    w_var(w, r_ncomp[r]);
  }
  for (uint32_t j = r0; j < r1; j++) {
    bool tail = j + 1 == NL || (cmp_head[j + 1] & 1);
    if (!tail) continue;
    uint32_t c = (uint32_t)(dkey[j] >> 32);
    // rank of c (binary search over d_client, ascending)
    uint32_t lo = 0, hi = D;
    while (lo < hi) {
      uint32_t mid = (lo + hi) / 2;
      if (d_client[mid] < c) lo = mid + 1;
      else hi = mid;
    }
    uint32_t r = lo;
    uint32_t hdr = varlen(c) + varlen(r_ncomp[r]);
    Writer w{dso, r_off[r] + hdr + (cmp_off[j] - cmp_off[r_beg[r]])};
    uint32_t cs = (uint32_t)dkey[j];
    w_var(w, cs);
    w_var(w, cmp_end[j] - cs);
  }
  if (t == 0) {
    o.path[d] = 0;
    o.status[d] = 0;
    o.out_len[d] = total;
    o.out_start[d] = slot;
  }
  YM_STAMP(11);
}

size_t fast_lds_bytes(const FastCaps &c) { return fast_layout(c).total; }

template <int NT> static void launch_nt(const BatchIn &b, const FastCaps &caps, const FastOut &o, size_t lds,
                                        hipStream_t s) {
  if (o.stamps) {
    hipFuncSetAttribute((const void *)k_fast_merge<NT, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((k_fast_merge<NT, true>), dim3(b.n_docs), dim3(NT), lds, s, b, caps, o);
  } else {
    hipFuncSetAttribute((const void *)k_fast_merge<NT, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((k_fast_merge<NT, false>), dim3(b.n_docs), dim3(NT), lds, s, b, caps, o);
  }
}

void launch_fast_merge(const BatchIn &b, const FastCaps &caps, const FastOut &o, int nt, hipStream_t s) {
  if (!b.n_docs) return;
  size_t lds = fast_lds_bytes(caps);
  if (nt == 1024)
    launch_nt<1024>(b, caps, o, lds, s);
  else if (nt == 512)
    launch_nt<512>(b, caps, o, lds, s);
  else
    launch_nt<256>(b, caps, o, lds, s);
}

} // namespace ym
