// ymerge_lean.hip — merge_updates_v1 for documents of the common editor shape: ONE
// WAVEFRONT per document, decode + placement + copy + DeleteSet union in a single pass,
// nothing round-tripped through HBM but the input and output bytes.
//
// Shape handled (everything else is handed to k_decode + k_fast_merge, path 3):
//   * every update is one client section with at most one block (Item with a Deleted or
//     ASCII String content, or a GC), or no section at all, plus a DeleteSet of at most 4
//     entries with distinct clients, non-empty ranges;
//   * per client, the blocks in input order are contiguous in clock (each starts where the
//     previous block of that client ended) — exactly the logs a sync server accumulates
//     from editors that ship one transaction per update;
//   * <= 16 distinct clients, document < 64 KB, every block < 1 KB, canonical encodings.
// For such a document yrs' merge (yrs/src/update.rs:537-704) reduces to: clients in
// descending order, each client's blocks verbatim in input order behind one section
// header (count, client, first clock), then the union of all DeleteSets
// (id_set.rs:129-164, 385-395) in the hashbrown order of first insertion
// (update.rs:542-548, std HashMap + ClientHasher).  Nothing is sorted, split or squashed.
//
// Per document (one wave, 64 lanes, no s_barrier):
//   1 decode, rounds of <= 64 updates: the round's bytes are staged into LDS with 16-byte
//     loads (the next round's bytes and offsets are already in flight), each lane walks one
//     update (ylds.h branch-free varints); clients -> buckets (LDS hash); per bucket the
//     contiguity check (ballot over the bucket's lanes, predecessor's end by lane shuffle),
//     counts and byte totals (LDS atomics); a 4-byte record per block (doc-relative source
//     offset, byte length, bucket); DeleteSet ranges to the top of the same arena.
//   2 layout: section order (client desc) and starts, section headers written.
//   3 copy: blocks in input order, <= 64 per step: their source bytes staged again with
//     16-byte loads, per-bucket prefix of byte lengths -> destination, LDS -> HBM stores
//     (dword stores for the aligned middle, byte stores at the two ends).
//   4 DeleteSet: bitmap union per client window in LDS (the arena is free by now), runs ->
//     components, sizes, hashbrown client order (one lane, <= 16 clients), write.
#include "ycodec.h"
#include "ykernels.h"
#include "ylds.h"
#include "ywalk.h"
#include "ywave.h"

namespace ym {

#ifndef YM_LN_STAGE
#define YM_LN_STAGE 2048
#endif
constexpr uint32_t LN_STAGE = YM_LN_STAGE; // staged bytes per round / copy step (2048: a C2 round takes 64
                                           // updates, 1536 took ~57: -7% k_lean)
static_assert(LN_STAGE < 65536, "copy phase: 16-bit per-bucket byte sums");
constexpr uint32_t LN_SW = LN_STAGE / 4 + 4; // stage words (+ the word after the last one lvar reads)
constexpr uint32_t LN_AW = 1280;             // arena words: block records grow up, DS ranges down
constexpr uint32_t LN_BUF = LN_SW + LN_AW;   // stage + arena, reused whole by the DeleteSet phase
constexpr uint32_t LN_NBK = 16;              // client buckets per document
constexpr uint32_t LN_MAXBLEN = 1024;        // block bytes (a copy step must always fit one block)
constexpr uint32_t LN_DSMAXI = 252;          // bytes of one update's DeleteSet
constexpr uint32_t LN_DSW = 1024;            // DeleteSet batch window: 16 staged bytes per lane
constexpr uint32_t LN_ORD = LN_NBK;          // DeleteSet entry offsets (end of buf, after the scatter)
constexpr uint32_t LN_NONE = 0xFFFFFFFFu;
constexpr uint32_t LN_UMAX = 16384;          // BIG documents: above, the grid path / tiled kernel (a 20k-update
                                             // trace document held one wave 0.43 ms before a hand-over)

// buf = [stage | arena]: block records (src | blen << 16 | bucket << 27) from the arena
// bottom; from the top, one word per DeleteSet item: its end offset in the document's DS
// scratch (the items themselves are copied verbatim to HBM, see phase 1).
struct LeanLds {
  uint32_t buf[LN_BUF];
  // per-bucket values updated by LDS atomics from many lanes; the rest of the per-bucket
  // state is register-resident (lane b = bucket b: client, first / next clock, copy cursor)
  uint32_t bytes[LN_NBK], dsfirst[LN_NBK];
};

// ------------------------------------------------------------------ one update
struct LeanUpd {
  uint32_t has_blk, client, clock, len, bpos, blen; // block; bpos = stage byte position
  uint32_t dspos, nent;                             // DeleteSet: stage position (its nds varint), entries
};

// Validating walk of one staged update (Update::decode_v1, yrs/src/update.rs:714-749,
// decode_block :433-488, ItemContent::decode block.rs:1786-1835) restricted to the lean
// shape; false = not the shape (or malformed: the exact walk downstream owns the error
// codes).  Straight-line with an accumulated `ok` (no early exits): lanes of one shape stay
// converged.  The DeleteSet is only located here (its entry count read); phase 4 decodes it.
YM_INLINE bool lean_walk(const uint32_t *w, uint32_t p, uint32_t n, LeanUpd &r) {
  const uint32_t end = p + n;
  r.has_blk = 0;
  r.nent = 0;
  const VarR ncl = var_at(w, p, end);
  bool ok = ncl.fine && ncl.v <= 1;
  p += ncl.n;
  if (ok && ncl.v == 1) {
    const VarR nb = var_at(w, p, end);
    const VarR cl = var_at(w, p + nb.n, end);
    const VarR ck = var_at(w, p + nb.n + cl.n, end);
    ok = nb.fine && cl.fine && ck.fine && nb.v <= 1;
    p += nb.n + cl.n + ck.n;
    if (ok && nb.v == 1) {
      const uint32_t bpos = p;
      const uint32_t info = lds_byte(w, p);
      p++;
      uint32_t len = 0;
      bool keep = true;
      if (info == 0 || info == 10) { // GC / Skip: canonical non-zero length
        const VarR l = var_at(w, p, end);
        ok = l.fine && l.canon && l.v != 0;
        p += l.n;
        len = l.v;
        keep = info == 0; // a Skip is dropped by IntoBlocks (update.rs:1054)
      } else {
        // origin / right origin (ID = 2 varints each), canonical: the block is copied verbatim
        if (info & 0x80) {
          const VarR a0 = var_at(w, p, end), a1 = var_at(w, p + a0.n, end);
          ok = ok && a0.fine && a0.canon && a1.fine && a1.canon;
          p += a0.n + a1.n;
        }
        if (info & 0x40) {
          const VarR a0 = var_at(w, p, end), a1 = var_at(w, p + a0.n, end);
          ok = ok && a0.fine && a0.canon && a1.fine && a1.canon;
          p += a0.n + a1.n;
        }
        uint32_t want = info & 0xCF;
        if ((info & 0xC0) == 0) { // parent: named root type (1) or ID (0), then parent_sub
          const VarR pi = var_at(w, p, end), x = var_at(w, p + pi.n, end);
          ok = ok && pi.fine && pi.canon && pi.v <= 1 && x.fine && x.canon;
          p += pi.n + x.n;
          if (pi.v == 1) {
            ok = ok && x.v <= end - p;
            p += x.v;
          } else {
            const VarR y = var_at(w, p, end);
            ok = ok && y.fine && y.canon;
            p += y.n;
          }
          if (info & 0x20) {
            want |= 0x20;
            const VarR sl = var_at(w, p, end);
            ok = ok && sl.fine && sl.canon && sl.v <= end - (p + sl.n);
            p += sl.n + sl.v;
          }
        }
        const uint32_t ref = info & 15;
        const VarR c = var_at(w, p, end);
        ok = ok && want == info && (ref == 1 || ref == 4) && c.fine && c.canon;
        p += c.n;
        len = c.v;
        if (ok && ref == 4) { // String: UTF-16 length == byte length for ASCII only
          ok = c.v <= end - p;
          const uint32_t s0 = p;
          p += c.v;
          if (ok && c.v > 1) {
            uint32_t hi = 0;
            const uint32_t e0 = s0 + c.v, q0 = s0 >> 2, q1 = (e0 - 1) >> 2;
            for (uint32_t q = q0; q <= q1; q++) {
              uint32_t x = w[q];
              if (q == q0) x &= 0xFFFFFFFFu << (8 * (s0 & 3));
              if (q == q1 && (e0 & 3)) x &= 0xFFFFFFFFu >> (8 * (4 - (e0 & 3)));
              hi |= x;
            }
            ok = !(hi & 0x80808080u);
          }
        }
        keep = len != 0; // Item::new drops zero-length items
      }
      ok = ok && p <= end;
      if (ok && keep) {
        ok = (uint64_t)ck.v + len <= 0xFFFFFFFFull && p - bpos <= LN_MAXBLEN;
        r.has_blk = 1;
        r.client = cl.v;
        r.clock = ck.v;
        r.len = len;
        r.bpos = bpos;
        r.blen = p - bpos;
      }
    }
  }
  r.dspos = p;
  const VarR nds = var_at(w, p, end);
  r.nent = nds.v;
  return ok && nds.fine && nds.v <= 4;
}

YM_INLINE uint32_t sel4(uint32_t i, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return i == 0 ? a : i == 1 ? b : i == 2 ? c : d;
}
// Iteration positions of <= 4 distinct DeleteSet entries in their update's HashMap
// (IdSet::decode inserts each in stream order; reserve(1) grows 0 -> 4 -> 8 buckets and
// re-places the old entries in slot order) — ds_order_packed (ywalk.h) in registers.
YM_INLINE void ds_pos4(uint32_t n, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t &p0, uint32_t &p1,
                       uint32_t &p2, uint32_t &p3) {
  uint64_t map = 0;
  uint32_t buckets = 0, items = 0, growth = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (growth == 0) {
      const uint32_t full = buckets ? (uint32_t)mask_to_cap(buckets - 1) : 0;
      const uint32_t need = items + 1;
      const uint32_t nb = (uint32_t)cap_to_buckets(need > full + 1 ? need : full + 1);
      uint64_t nm = 0;
      for (uint32_t s = 0; s < buckets; s++) {
        const uint32_t en = (uint32_t)(map >> (4 * s)) & 15;
        if (en) nm |= (uint64_t)en << (4 * hb_probe(nm, nb, sel4(en - 1, c0, c1, c2, c3)));
      }
      map = nm;
      buckets = nb;
      growth = (uint32_t)mask_to_cap(nb - 1) - items;
    }
    map |= (uint64_t)(i + 1) << (4 * hb_probe(map, buckets, sel4(i, c0, c1, c2, c3)));
    items++;
    growth--;
  }
  uint32_t k = 0;
  p0 = p1 = p2 = p3 = 0;
  for (uint32_t s = 0; s < buckets; s++) {
    const uint32_t en = (uint32_t)(map >> (4 * s)) & 15;
    if (en == 1) p0 = k++;
    else if (en == 2) p1 = k++;
    else if (en == 3) p2 = k++;
    else if (en == 4) p3 = k++;
  }
}

// ------------------------------------------------------------------ client buckets
// Client buckets live in registers: lane b of `tabc` holds the client of bucket b < nbk
// (wave-uniform count), so a lookup is nbk readlane + compare steps, no memory round trip.
YM_INLINE int tab_find(uint32_t tabc, uint32_t nbk, uint32_t c) {
  int r = -1;
  for (uint32_t q = 0; q < nbk; q++) r = rdlane(tabc, q) == c ? (int)q : r;
  return r;
}
// bucket of client c for the lanes with `want`; unknown clients are appended one per
// iteration (uniform loop).  false = more than LN_NBK clients.
YM_INLINE bool bucket_of(uint32_t lane, uint32_t &tabc, uint32_t c, bool want, uint32_t &nbk, int &bk) {
  bk = want ? tab_find(tabc, nbk, c) : 0;
  for (;;) {
    const uint64_t m = __ballot(want && bk < 0);
    if (!m) return true;
    if (nbk == LN_NBK) return false;
    const uint32_t cn = rdlane(c, (uint32_t)__builtin_ctzll(m));
    if (lane == nbk) tabc = cn;
    if (want && bk < 0 && c == cn) bk = (int)nbk;
    nbk++;
  }
}

// ------------------------------------------------------------------ LDS -> HBM byte copy
// n bytes from staged byte position so to dp: byte stores up to dp's dword alignment, dword
// stores (two staged dwords aligned by v_alignbyte) for the middle, byte stores for the tail.
YM_INLINE void copy_out(const uint32_t *st, uint32_t so, uint8_t *dp, uint32_t n) {
  const uint8_t *sb = (const uint8_t *)st;
  uint32_t head = (uint32_t)(0u - (uint32_t)(uintptr_t)dp) & 3u;
  if (head > n) head = n;
  for (uint32_t q = 0; q < head; q++) dp[q] = sb[so + q];
  uint32_t p = so + head, rem = n - head;
  uint8_t *dq = dp + head;
  if (rem >= 4) {
    const uint32_t sh = p & 3;
    uint32_t q4 = p >> 2, lo = st[q4];
    for (; rem >= 4; rem -= 4) {
      const uint32_t hi = st[++q4];
      *(uint32_t *)dq = __builtin_amdgcn_alignbyte(hi, lo, sh);
      lo = hi;
      dq += 4;
      p += 4;
    }
  }
  for (uint32_t q = 0; q < rem; q++) dq[q] = sb[p + q];
}

// n bytes LDS -> LDS (byte positions sp -> dp): byte stores up to dp's dword alignment and
// for the tail, dword stores (v_alignbyte of two source dwords) between
YM_INLINE void copy_lds(const uint32_t *sw, uint32_t sp, uint32_t *dw, uint32_t dp, uint32_t n) {
  const uint8_t *sb = (const uint8_t *)sw;
  uint8_t *db = (uint8_t *)dw;
  uint32_t head = (4u - (dp & 3)) & 3u;
  if (head > n) head = n;
  for (uint32_t q = 0; q < head; q++) db[dp + q] = sb[sp + q];
  uint32_t p = sp + head, d = dp + head, rem = n - head;
  if (rem >= 4) {
    const uint32_t sh = p & 3;
    uint32_t q4 = p >> 2, lo = sw[q4];
    for (; rem >= 4; rem -= 4) {
      const uint32_t hi = sw[++q4];
      dw[d >> 2] = __builtin_amdgcn_alignbyte(hi, lo, sh);
      lo = hi;
      d += 4;
      p += 4;
    }
  }
  for (uint32_t q = 0; q < rem; q++) db[d + q] = sb[p + q];
}

// 16-byte staging of absolute bytes [al, al + 16 * n16) (n16 <= LN_STAGE / 16) into buf
YM_INLINE void stage_load(const uint8_t *bytes, uint64_t al, uint32_t n16, uint32_t lane, uint4 &v0, uint4 &v1) {
  const uint4 *src = (const uint4 *)(bytes + al);
  if (lane < n16) v0 = src[lane];
  if (lane + 64 < n16) v1 = src[lane + 64];
}
YM_INLINE void stage_store(uint32_t *buf, uint32_t n16, uint32_t lane, const uint4 &v0, const uint4 &v1) {
  if (lane < n16) ((uint4 *)buf)[lane] = v0;
  if (lane + 64 < n16) ((uint4 *)buf)[lane + 64] = v1;
}

// DeleteSet client order: IdSet::merge (id_set.rs:385-395) inserts the clients of every
// update's table into the result table in first-occurrence order (update.rs:542-548);
// std's hashbrown with the identity ClientHasher (utils/client_hasher.rs) then iterates
// in slot order.  Restated as k_fast_merge's emulation (ymerge_fast.hip, phase 5b) for
// <= LN_NBK clients, with the table in registers (lane s = slot s < 32, bucket + 1 or 0),
// computed by the whole wave (uniform control): a probe is one lane shuffle + ballot over
// the 16 control bytes of the group (round 5: one lane, 16 dependent LDS reads per probe,
// 5 % of k_lean on C2).  Lane b (a
// bucket with a DeleteSet entry: hasd) gets its entry's offset; `total` = the end.
YM_INLINE uint32_t lean_ds_order_wave(uint32_t lane, uint32_t nbk, bool hasd, uint32_t dsf, uint32_t cl,
                                      uint32_t esz, uint32_t start, uint32_t *eoff, uint32_t &total) {
  const uint64_t hm = __ballot(hasd);
  const uint32_t D = (uint32_t)__builtin_popcountll(hm);
  uint32_t rank = 0; // insertion order: first occurrence (dsfirst values are distinct)
  for (uint32_t q = 0; q < nbk; q++) {
    const uint32_t fq = rdlane(dsf, q);
    rank += (((hm >> q) & 1) && fq < dsf) ? 1u : 0u;
  }
  uint32_t slotv = 0, buckets = 0, items = 0, growth = 0;
  auto find_slot = [&](uint32_t key) -> uint32_t {
    const uint32_t mask = buckets - 1;
    uint32_t pos = key & mask, stride = 0;
    for (;;) {
      // ctrl_empty(pos + j) for j = lane < 16 (hashbrown's group probe): real slots, then the
      // trailing control bytes (EMPTY beyond a small table's mirror)
      const uint32_t idx = pos + (lane & 15);
      const uint32_t si = idx < buckets ? idx : buckets < 16 ? idx - 16 : idx - buckets;
      const uint32_t sv = shfl(slotv, (int)(si & 63));
      const bool emp = idx < buckets ? sv == 0 : buckets < 16 ? (idx < 16 || sv == 0) : sv == 0;
      const uint64_t em = __ballot(lane < 16 && emp);
      if (em) {
        const uint32_t index = (pos + (uint32_t)__builtin_ctzll(em)) & mask;
        if (rdlane(slotv, index) != 0) return (uint32_t)__builtin_ctzll(__ballot(lane < buckets && slotv == 0));
        return index;
      }
      stride += 16;
      pos = (pos + stride) & mask;
    }
  };
  for (uint32_t i = 0; i < D; i++) {
    if (growth == 0) {
      const uint64_t full = buckets ? mask_to_cap(buckets - 1) : 0;
      const uint64_t need = items + 1;
      const uint32_t nb = (uint32_t)cap_to_buckets(need > full + 1 ? need : full + 1); // <= 32 for 16 items
      const uint32_t ob = buckets, tmpv = slotv;
      buckets = nb;
      slotv = 0;
      for (uint32_t q = 0; q < ob; q++) {
        const uint32_t t = rdlane(tmpv, q);
        if (t) {
          const uint32_t sl = find_slot(rdlane(cl, t - 1));
          if (lane == sl) slotv = t;
        }
      }
      growth = (uint32_t)mask_to_cap(buckets - 1) - items;
    }
    const uint32_t bq = (uint32_t)__builtin_ctzll(__ballot(hasd && rank == i));
    const uint32_t sl = find_slot(rdlane(cl, bq));
    if (lane == sl) slotv = bq + 1;
    items++;
    growth--;
  }
  // entries in slot order: offsets by a prefix over the slots, scattered to their buckets
  const bool occ = slotv != 0;
  const uint32_t sz = shfl(esz, (int)(occ ? slotv - 1 : 0));
  const uint32_t mine = occ ? sz : 0u;
  const uint32_t inc = wincl(mine, lane);
  total = start + rdlane(inc, 63);
  if (occ) eoff[slotv - 1] = start + inc - mine;
  wsync();
  return hasd ? eoff[lane] : 0u;
}

// ------------------------------------------------------------------ the kernel
// Diagnostic build only (STAMPS, env YMERGE_STAMPS): lane 0 records s_memtime at phase
// boundaries into o.stamps[doc * 16 + k] (k 0..6), per-round sub-phase cycle sums (8..11),
// rounds (12), marker 0x1EA4 (15); never part of a timed run.
// BIG (documents above the LDS arena: > LN_AW updates or >= 64 KB): the same algorithm
// with the size-proportional tables in the document's HBM scratch `scr` (word offset
// 4 * u0 + 64 * d + B0, capacity 4 U + 64 + bytes words): block records (2 words) at
// [0, 2U), DeleteSet item ends at [2U, 3U), the DeleteSet bitmap from 3U, component starts /
// ends after it.  LDS then holds only the stage and the DeleteSet batch.
// YM_LEAN_STOP=k (diagnostic builds only, tools/lean_phases.sh): end every document after
// phase k (1 decode, 2 layout, 3 copy, 4 DeleteSet scatter, 5 components, 6 client order)
// with an empty result, so that per-phase instruction
// counts can be read from the SQ counters as differences
#ifdef YM_LEAN_STOP
#define LEAN_STOP(k)                                                                                                   \
  if (YM_LEAN_STOP == (k)) {                                                                                           \
    if (lane == 0) {                                                                                                   \
      o.path[d] = 0;                                                                                                   \
      o.status[d] = 0;                                                                                                 \
      o.out_len[d] = 0;                                                                                                \
      o.out_start[d] = slot;                                                                                           \
    }                                                                                                                  \
    return;                                                                                                            \
  }
#else
#define LEAN_STOP(k)
#endif
template <bool BIG, bool STAMPS>
__device__ __forceinline__ void lean_doc(const BatchIn &b, const FastOut &o, LeanLds &L, const uint32_t d,
                                         const uint32_t lane, uint32_t *const scr) {
  uint64_t tst[16];
  auto stamp = [&](int k) {
    if (STAMPS) tst[k] = __builtin_amdgcn_s_memtime();
  };
  auto acc = [&](int k, uint64_t t0) {
    if (STAMPS) tst[k] += __builtin_amdgcn_s_memtime() - t0;
  };
  if (STAMPS)
    for (int q = 0; q < 16; q++) tst[q] = 0;
  stamp(0);
  const uint64_t u0 = b.doc_upd[d], u1 = b.doc_upd[d + 1];
  const uint64_t B0 = b.upd_off[u0], B1 = b.upd_off[u1];
  const uint32_t U = (uint32_t)(u1 - u0);
  const uint64_t slot = 2 * B0 + 64ull * d;
  uint8_t *out = o.out + slot;
  // hand-over; why: 0 size/empty, 1 stage, 2 walk, 3 clients, 4 arena, 5 contiguity, 6 DS window
  // (npath[7 + why]: diagnostics, env YMERGE_LEAN_DEBUG)
  // The count goes to this document's shard (word 2 of its 64-byte output-byte partial,
  // summed by k_lean_fin / the host): one counter for every handing-over wave serialised the
  // corpus's 78 k hand-overs on one address (k_lean 1.53 ms, §5.10).
  auto reject = [&](uint32_t why) {
    if (lane == 0) {
      o.path[d] = 3;
      if (o.lean_total) atomicAdd((uint32_t *)(o.lean_total + 8 * (d & 63)) + 2, 1u);
      else atomicAdd(&o.npath[6], 1u);
      if (o.dbg) atomicAdd(&o.npath[7 + (why < 7 ? why : 0)], 1u);
    }
  };
  if (U == 0 || (!BIG && (B1 - B0 >= 65536 || U > LN_AW))) {
    reject(0);
    return;
  }
  // this document's HBM scratch (every document has one when scr is set; BIG documents
  // keep all their tables there, the others only component lists that outgrow LDS)
  uint32_t *const hs = scr ? scr + 4 * u0 + 64ull * d + B0 : nullptr;
  auto item_end = [&](uint32_t j) -> uint32_t { return BIG ? hs[2 * U + j] : L.buf[LN_BUF - 1 - j]; };
  if (lane < LN_NBK) {
    L.bytes[lane] = 0;
    L.dsfirst[lane] = LN_NONE;
  }
  wsync();

  // ---------------------------------------------------------------- 1 decode
  uint32_t nbk = 0, NBk = 0, NI = 0, blkmask = 0;
  // DeleteSet scratch: the upper half of this document's output slot (capacity 2 x input +
  // 64; a lean document's output is at most its input + 10 bytes), DSB bytes used
  uint8_t *const dscr = out + (B1 - B0) + 64;
  uint32_t DSB = 0;
  // per bucket (lane = bucket): client, first / next clock, block count
  uint32_t tabc = 0, bfirst = 0, bnext = 0, bcnt = 0;
  uint32_t bad = 0; // why + 1
  uint32_t ub = 0;
  uint64_t A = B0;
  // round pipeline: offsets of the round's updates (e = end of update ub + lane), its
  // staged bytes; the next round's are loaded while this one is walked
  uint64_t e = lane < U ? b.upd_off[u0 + 1 + lane] : 0;
  uint64_t en = lane + 64 < U ? b.upd_off[u0 + 65 + lane] : 0; // the 64 after
  uint32_t k, n16;
  uint64_t al = A & ~15ull, E;
  {
    const uint64_t fm = __ballot(lane < U && e - al <= LN_STAGE);
    k = lead_ones(fm);
    if (k == 0) {
      reject(1);
      return;
    }
    E = rdlane64(e, k - 1);
    n16 = (uint32_t)((E - al + 15) >> 4);
  }
  uint4 v0, v1;
  stage_load(b.bytes, al, n16, lane, v0, v1);
  stamp(1);
  while (ub < U) {
    const uint64_t tr0 = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    if (STAMPS) tst[12]++;
    const uint64_t sprev = shfl(e, lane ? (int)lane - 1 : 0); // every lane takes part in the shuffle
    const uint64_t s = lane == 0 ? A : sprev;
    const bool act = lane < k;
    const uint32_t i = ub + lane; // doc-relative update index
    stage_store(L.buf, n16, lane, v0, v1);
    // next round: shift the offset window by k, load the next offsets and bytes
    const uint32_t ub2 = ub + k;
    const uint64_t A2 = E;
    uint64_t e2 = 0, en2 = 0;
    uint32_t k2 = 0, n162 = 0;
    uint64_t al2 = A2 & ~15ull, E2 = A2;
    if (ub2 < U) {
      // e2 = end of update ub2 + lane: from this round's window (e: ub.., en: ub + 64..)
      const uint32_t sl = (lane + k) & 63;
      const uint64_t x = shfl(e, (int)sl), y = shfl(en, (int)sl);
      e2 = lane + k < 64 ? x : y;
      // en2 = end of update ub2 + 64 + lane: loaded now, needed one round later
      const uint32_t gi = ub2 + 64 + lane;
      en2 = gi < U ? b.upd_off[u0 + 1 + gi] : 0;
      const uint64_t fm = __ballot(ub2 + lane < U && e2 - al2 <= LN_STAGE);
      k2 = lead_ones(fm);
      if (k2 > 0) {
        E2 = rdlane64(e2, k2 - 1);
        n162 = (uint32_t)((E2 - al2 + 15) >> 4);
      }
    }
    uint4 w0 = make_uint4(0, 0, 0, 0), w1 = w0;
    if (k2 > 0) stage_load(b.bytes, al2, n162, lane, w0, w1);
    wsync();
    acc(8, tr0);
    const uint64_t tr1 = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    // walk this round's updates
    LeanUpd r;
    bool ok = true;
    r.has_blk = r.nent = 0;
    r.client = r.clock = r.len = r.bpos = r.blen = r.dspos = 0;
    if (act) ok = lean_walk(L.buf, (uint32_t)(s - al), (uint32_t)(e - s), r);
    if (__ballot(act && !ok)) {
      bad = 3;
      break;
    }
    acc(9, tr1);
    const uint64_t tr2 = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    // blocks: buckets, contiguity, counts, records
    const bool hb = act && r.has_blk;
    int bk;
    if (!bucket_of(lane, tabc, r.client, hb, nbk, bk)) {
      bad = 4;
      break;
    }
    const uint64_t mall = __ballot(hb);
    const uint32_t nbr = (uint32_t)__builtin_popcountll(mall);
    if (!BIG && NBk + nbr + NI > LN_AW) { // arena full: not lean
      bad = 5;
      break;
    }
    if (mall) {
      int prevl = -1;
      uint32_t exp0 = 0;
      uint64_t rem = mall;
      const uint32_t endv = r.clock + r.len;
      while (rem) {
        const uint32_t lead = (uint32_t)__builtin_ctzll(rem);
        const uint32_t bb = rdlane((uint32_t)bk, lead);
        const uint64_t mb = __ballot(hb && (uint32_t)bk == bb);
        rem &= ~mb;
        const uint32_t last = 63 - (uint32_t)__builtin_clzll(mb);
        const uint32_t c0 = rdlane(r.clock, lead), nend = rdlane(endv, last);
        const bool had = (blkmask >> bb) & 1;
        const uint32_t nxt = had ? rdlane(bnext, bb) : c0;
        if (hb && (uint32_t)bk == bb) {
          const uint64_t lt = mb & ((1ull << lane) - 1);
          prevl = lt ? 63 - (int)__builtin_clzll(lt) : -1;
          exp0 = nxt;
        }
        if (lane == bb) {
          if (!had) bfirst = c0;
          bnext = nend;
          bcnt += (uint32_t)__builtin_popcountll(mb);
        }
        blkmask |= 1u << bb;
      }
      const uint32_t pend = shfl(endv, prevl < 0 ? (int)lane : prevl);
      const bool okc = !hb || r.clock == (prevl < 0 ? exp0 : pend);
      if (__ballot(!okc)) {
        bad = 6;
        break;
      }
      if (hb) {
        atomicAdd(&L.bytes[bk], r.blen);
        const uint32_t src = (uint32_t)(al + r.bpos - B0), ri = NBk + lanes_below(mall);
        if (BIG) {
          hs[2 * ri] = src;
          hs[2 * ri + 1] = r.blen | ((uint32_t)bk << 27);
        } else {
          L.buf[LN_SW + ri] = src | (r.blen << 16) | ((uint32_t)bk << 27);
        }
      }
      NBk += nbr;
    }
    acc(10, tr2);
    const uint64_t tr3 = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    // DeleteSets: item bytes verbatim to the HBM scratch (input order), end offsets to the
    // arena top; decoded in a few large batches by phase 4
    {
      const bool hd = act && r.nent > 0;
      const uint32_t ilen = hd ? (uint32_t)(e - al) - r.dspos : 0;
      const uint64_t hm = __ballot(hd);
      if (hm) {
        const uint32_t binc = wincl(ilen, lane), btot = rdlane(binc, 63);
        const uint32_t nit = (uint32_t)__builtin_popcountll(hm);
        if (__ballot(ilen > LN_DSMAXI)) {
          bad = 3;
          break;
        }
        if (!BIG && NBk + NI + nit > LN_AW) {
          bad = 5;
          break;
        }
        if (hd) {
          copy_out(L.buf, r.dspos, dscr + DSB + binc - ilen, ilen);
          const uint32_t ii = NI + lanes_below(hm);
          if (BIG) hs[2 * U + ii] = DSB + binc;
          else L.buf[LN_BUF - 1 - ii] = DSB + binc;
        }
        NI += nit;
        DSB += btot;
      }
    }
    acc(11, tr3);
    // advance
    ub = ub2;
    A = A2;
    e = e2;
    en = en2;
    if (ub < U && k2 == 0) { // one update larger than the stage: not lean
      bad = 2;
      break;
    }
    k = k2;
    n16 = n162;
    al = al2;
    E = E2;
    v0 = w0;
    v1 = w1;
    wsync();
  }
  if (bad) {
    reject(bad - 1);
    return;
  }
  wsync();
  stamp(2);
  LEAN_STOP(1)

  // ---------------------------------------------------------------- 2 layout
  const bool lb = lane < nbk;
  const uint32_t cnt = lb ? bcnt : 0, cl = lb ? tabc : 0, fst = lb ? bfirst : 0, byt = lb ? L.bytes[lane] : 0;
  const bool hasb = cnt > 0;
  const uint64_t hbm = __ballot(hasb);
  const uint32_t NC = (uint32_t)__builtin_popcountll(hbm);
  uint32_t rank = 0;
  for (uint32_t q = 0; q < nbk; q++) {
    const uint32_t cq = rdlane(cl, q);
    rank += (((hbm >> q) & 1) && cq > cl) ? 1u : 0u;
  }
  const uint32_t hdr = hasb ? varlen(cnt) + varlen(cl) + varlen(fst) : 0;
  const uint32_t ssz = hasb ? hdr + byt : 0;
  uint32_t sst = varlen(NC), blocks_size = varlen(NC);
  for (uint32_t q = 0; q < nbk; q++) {
    const uint32_t rq = rdlane(rank, q), sq = rdlane(ssz, q);
    blocks_size += sq;
    if (((hbm >> q) & 1) && rq < rank) sst += sq;
  }
  // DeleteSet bitmap: one window per client with blocks, [first clock & ~31, next clock) — a
  // lean DeleteSet deletes clocks of the document's own blocks (else: handed over)
  const uint32_t bnx = hasb ? bnext : 0;
  const uint32_t dbase = hasb ? fst & ~31u : 0;
  const uint32_t words = hasb ? ((bnx - 1) >> 5) - (dbase >> 5) + 1 : 0;
  const uint32_t win = wincl(words, lane), W = rdlane(win, 63), woff = win - words;
  const uint32_t Wr = (W + 3) & ~3u; // staging after the bitmap, 16-byte aligned
  // DS batches need the bitmap, a staging window and its decoded varints below the item ends.
  // The bitmap goes to the HBM scratch ([3U, 3U + Wr), then the component lists: 2 NR <= DSB
  // words, within the scratch's last U + 64 + bytes words) for BIG documents and whenever
  // it would leave no room for one batch of the largest item.
  const bool bmg = BIG || Wr + LN_DSW / 4 + 8 + LN_DSMAXI + NI > LN_BUF;
  const uint32_t lds_used = (BIG ? 0 : NI) + (bmg ? 0 : Wr);
  const uint32_t dsavail = LN_BUF - lds_used > LN_DSW / 4 + 8 ? LN_BUF - lds_used - (LN_DSW / 4 + 8) : 0;
  const uint32_t dslim = dsavail < LN_DSW - 16 ? dsavail : LN_DSW - 16; // batch bytes (<= varints)
  if ((NI && dslim < LN_DSMAXI) || (bmg && (!hs || (uint64_t)Wr + DSB > U + 64 + (B1 - B0)))) {
    reject(6);
    return;
  }
  // section headers (count, client, first clock: update.rs encode_diff :490-535) and NC
  if (lane == 0) {
    Writer wr{out, 0};
    w_var(wr, NC);
  }
  uint32_t curr = sst + hdr; // copy cursor of bucket `lane`
  if (hasb) {
    Writer wr{out, sst};
    w_var(wr, cnt);
    w_var(wr, cl);
    w_var(wr, fst);
  }
  wsync();

  LEAN_STOP(2)
  stamp(3);
  // ---------------------------------------------------------------- 3 copy blocks
  {
    uint32_t r0 = 0;
    uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0;
    uint32_t rsrc = 0, rmeta = 0, kk = 0, cn16 = 0; // record: source offset, blen | bucket << 27
    uint64_t cal = 0;
    auto plan = [&](uint32_t base) {
      const uint32_t j = base + lane;
      const bool v = j < NBk;
      if (BIG) {
        rsrc = v ? hs[2 * j] : 0;
        rmeta = v ? hs[2 * j + 1] : 0;
      } else {
        const uint32_t rec = v ? L.buf[LN_SW + j] : 0;
        rsrc = rec & 0xFFFF;
        rmeta = ((rec >> 16) & 0x7FF) | (rec & 0x78000000u);
      }
      const uint32_t src = rsrc, bl = rmeta & 0x7FF;
      cal = (B0 + rdlane(src, 0)) & ~15ull;
      const uint64_t ae = B0 + src + bl;
      kk = lead_ones(__ballot(v && ae - cal <= LN_STAGE));
      const uint64_t Ek = rdlane64(ae, kk - 1);
      cn16 = (uint32_t)((Ek - cal + 15) >> 4);
    };
    if (NBk) {
      plan(0);
      stage_load(b.bytes, cal, cn16, lane, c0, c1);
    }
    while (r0 < NBk) {
      const uint32_t mysrc = rsrc, mymeta = rmeta, k1 = kk, n1 = cn16;
      const uint64_t al1 = cal;
      stage_store(L.buf, n1, lane, c0, c1);
      const uint32_t r1 = r0 + k1;
      if (r1 < NBk) { // next step's plan and bytes in flight during this one
        plan(r1);
        stage_load(b.bytes, cal, cn16, lane, c0, c1);
      }
      wsync();
      const bool act = lane < k1;
      const uint32_t src = mysrc, bl = mymeta & 0x7FF, bq = (mymeta >> 27) & 15;
      uint32_t off = 0;
      if (nbk <= 4) {
        // <= 4 clients: the per-bucket prefix sums as 16-bit fields of two scans (a step's
        // blocks lie within LN_STAGE staged bytes, so no field carries)
        const uint32_t sh = 16 * (bq & 1);
        const uint32_t il = wincl(act && bq < 2 ? bl << sh : 0u, lane), ih = wincl(act && bq >= 2 ? bl << sh : 0u, lane);
        const uint32_t tl = rdlane(il, 63), th = rdlane(ih, 63);
        const uint32_t c0 = rdlane(curr, 0), c1 = rdlane(curr, 1), c2 = rdlane(curr, 2), c3 = rdlane(curr, 3);
        const uint32_t inc = ((bq < 2 ? il : ih) >> sh) & 0xFFFFu;
        if (act) off = (bq == 0 ? c0 : bq == 1 ? c1 : bq == 2 ? c2 : c3) + inc - bl;
        if (lane < 4) curr += ((lane < 2 ? tl : th) >> (16 * (lane & 1))) & 0xFFFFu;
      } else {
        uint64_t rem = __ballot(act);
        while (rem) {
          const uint32_t bb = rdlane(bq, (uint32_t)__builtin_ctzll(rem));
          const bool mine = act && bq == bb;
          rem &= ~__ballot(mine);
          const uint32_t inc = wincl(mine ? bl : 0u, lane), tot = rdlane(inc, 63);
          const uint32_t base = rdlane(curr, bb);
          if (mine) off = base + inc - bl;
          if (lane == bb) curr = base + tot;
        }
      }
      if (act) copy_out(L.buf, (uint32_t)(B0 + src - al1), out + off, bl);
      wsync();
      r0 = r1;
    }
  }

  LEAN_STOP(3)
  stamp(4);
  // ---------------------------------------------------------------- 4 DeleteSet
  // IdSet::decode of every item (id_set.rs:412-426) in batches of whole items staged from the
  // HBM scratch; ranges go straight into the bitmap (IdSet::merge + squash = union,
  // id_set.rs:129-164, 385-395); first-occurrence keys give the union's client order.
  uint32_t *const bmp = bmg ? hs + 3 * U : L.buf;
  for (uint32_t q = lane; q < W; q += 64) bmp[q] = 0;
  // the wave's scratch stores must be visible to its own loads below
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  wsync();
  uint32_t *const stg = bmg ? L.buf : L.buf + Wr, *const dsv = stg + LN_DSW / 4 + 8;
  uint32_t NR = 0; // ranges (bound the components)
  {
    const uint64_t tp0 = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t i0 = 0, s0 = 0;
    uint32_t dbad = 0; // why + 1
    while (i0 < NI && !dbad) {
      if (STAMPS) tst[14]++;
      // items [i0, i1) with their bytes [s0, s1) <= dslim (item ends are ascending)
      uint32_t i1 = i0;
      for (;;) {
        const uint32_t j = i1 + lane;
        const uint64_t fm = __ballot(j < NI && item_end(j) - s0 <= dslim);
        const uint32_t kf = lead_ones(fm);
        i1 += kf;
        if (kf < 64) break;
      }
      const uint32_t s1 = item_end(i1 - 1);
      const uint64_t ga = (uint64_t)(uintptr_t)(dscr + s0), ga16 = ga & ~15ull;
      const uint32_t so = (uint32_t)(ga - ga16), send = so + (s1 - s0);
      {
        uint4 d0 = make_uint4(0, 0, 0, 0), d1 = d0;
        const uint32_t n16 = (send + 15) >> 4;
        stage_load((const uint8_t *)(uintptr_t)ga16, 0, n16, lane, d0, d1);
        stage_store(stg, n16, lane, d0, d1);
      }
      wsync();
      // 1 terminators (bit 7 clear) of bytes [16 lane, 16 lane + 16) within [so, send); a
      // varint starts at so and after every terminator; its index = terminators before it
      const uint32_t b0 = 16 * lane;
      const uint32_t lo = so > b0 ? so - b0 : 0, hi = send > b0 ? send - b0 : 0;
      const uint32_t vmask = (hi >= 16 ? 0xFFFFu : (1u << hi) - 1) & ~(lo >= 16 ? 0xFFFFu : (1u << lo) - 1);
      uint32_t tm = 0;
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t t = ~stg[4 * lane + q] & 0x80808080u;
        tm |= (((t >> 7) & 1) | ((t >> 14) & 2) | ((t >> 21) & 4) | ((t >> 28) & 8)) << (4 * q);
      }
      tm &= vmask;
      const uint32_t ns = (uint32_t)__builtin_popcount(tm);
      const uint32_t ginc = wincl(ns, lane), gbase = ginc - ns;
      const uint32_t tprev = shfl(tm, lane ? (int)lane - 1 : 0);
      uint32_t sm = ((tm << 1) | (lane == 0 ? 1u << so : (tprev >> 15) & 1)) & vmask; // lane 0: the batch's first byte
      bool vok = true;
      while (sm) {
        const uint32_t kb = (uint32_t)__builtin_ctz(sm);
        const VarR r = var_at(stg, b0 + kb, send);
        vok = vok && r.fine;
        dsv[gbase + (uint32_t)__builtin_popcount(tm & ((1u << kb) - 1))] = r.v;
        sm &= sm - 1;
      }
      if (__ballot(!vok)) {
        dbad = 4;
        break;
      }
      wsync();
      // 2 one lane per item, groups of 64; entries in lockstep (uniform loop)
      for (uint32_t g0i = i0; g0i < i1 && !dbad; g0i += 64) {
        const uint32_t it = g0i + lane;
        const bool iv = it < i1;
        const uint32_t ist = iv ? (it ? item_end(it - 1) : 0) - s0 + so : so;
        const uint32_t ien = iv ? item_end(it) - s0 + so : so + 1;
        const uint32_t ja = ist >> 4, jz = (ien - 1) >> 4;
        const uint32_t gba = shfl(gbase, (int)(ja & 63)), tma = shfl(tm, (int)(ja & 63));
        const uint32_t gbz = shfl(gbase, (int)(jz & 63)), tmz = shfl(tm, (int)(jz & 63));
        const uint32_t g0 = gba + (uint32_t)__builtin_popcount(tma & ((1u << (ist & 15)) - 1));
        const uint32_t zb = (ien - 1) & 15;
        const uint32_t gend = gbz + (uint32_t)__builtin_popcount(tmz & ((2u << zb) - 1));
        bool ok = !iv || ((tmz >> zb) & 1); // the item's last byte ends a varint
        const uint32_t nds = iv ? dsv[g0] : 0;
        ok = ok && (!iv || (nds >= 1 && nds <= 4 && g0 < gend));
        const uint32_t nent = iv && ok ? nds : 0;
        uint32_t g = g0 + 1, nrec = 0;
        uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
        int b0k = 0, b1k = 0, b2k = 0, b3k = 0;
#pragma unroll
        for (uint32_t e = 0; e < 4; e++) {
          bool ae = ok && e < nent;
          if (!__ballot(ae)) break;
          uint32_t cv = 0, nr = 0;
          if (ae) {
            ae = g + 2 <= gend;
            if (ae) {
              cv = dsv[g];
              nr = dsv[g + 1];
              ae = nr >= 1 && nr <= ien - ist && g + 2 + 2 * nr <= gend && !(e > 0 && c0 == cv) &&
                   !(e > 1 && c1 == cv) && !(e > 2 && c2 == cv);
            }
          }
          // the entry's client must own blocks here (its window): else not lean
          const int bq = ae ? tab_find(tabc, nbk, cv) : 0;
          ae = ae && bq >= 0 && ((blkmask >> (bq & 31)) & 1);
          const uint32_t bqq = (uint32_t)(bq < 0 ? 0 : bq) & 63;
          const uint32_t f0 = shfl(fst, (int)bqq), bn = shfl(bnx, (int)bqq);
          const uint32_t wo = shfl(woff, (int)bqq), bs = shfl(dbase, (int)bqq);
          if (e == 0) { c0 = cv; b0k = bq; }
          else if (e == 1) { c1 = cv; b1k = bq; }
          else if (e == 2) { c2 = cv; b2k = bq; }
          else { c3 = cv; b3k = bq; }
          if (ae) {
            for (uint32_t t = 0; t < nr && ae; t++) {
              const uint32_t a = dsv[g + 2 + 2 * t], l = dsv[g + 3 + 2 * t];
              ae = l != 0 && a >= f0 && (uint64_t)a + l <= bn;
              if (!ae) break;
              uint32_t x = a - bs;
              const uint32_t z = x + l;
              while (x < z) {
                const uint32_t wi = x >> 5, bo = x & 31, nb = (z - x < 32 - bo) ? z - x : 32 - bo;
                const uint32_t mask = (nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1)) << bo;
                atomicOr(&bmp[wo + wi], mask);
                x += nb;
              }
            }
            nrec += nr;
            g += 2 + 2 * nr;
          }
          if (e < nent) ok = ae;
        }
        ok = ok && (!iv || g == gend); // no varints after the DeleteSet (trailing bytes: not lean)
        if (__ballot(iv && !ok)) {
          dbad = 7; // window (a range outside its client's blocks) or malformed: hand over
          break;
        }
        if (iv) {
          uint32_t p0 = 0, p1 = 1, p2 = 2, p3 = 3;
          if (nent >= 2) ds_pos4(nent, c0, c1, c2, c3, p0, p1, p2, p3);
          atomicMin(&L.dsfirst[b0k], (it << 8) | p0);
          if (nent > 1) atomicMin(&L.dsfirst[b1k], (it << 8) | p1);
          if (nent > 2) atomicMin(&L.dsfirst[b2k], (it << 8) | p2);
          if (nent > 3) atomicMin(&L.dsfirst[b3k], (it << 8) | p3);
        }
        NR += rdlane(wincl(nrec, lane), 63);
      }
      wsync();
      i0 = i1;
      s0 = s1;
    }
    acc(13, tp0);
    if (dbad) {
      reject(dbad - 1);
      return;
    }
  }
  LEAN_STOP(4)
  const uint32_t dsf = lb ? L.dsfirst[lane] : LN_NONE;
  const bool hasd = dsf != LN_NONE;
  const uint32_t D = (uint32_t)__builtin_popcountll(__ballot(hasd));
  // component starts / ends: LDS after the bitmap when they fit below the order scratch,
  // else the scratch after the bitmap's region (2 NR <= DeleteSet bytes <= input)
  const bool cg = bmg || W + 2 * NR + LN_ORD > LN_BUF;
  if (cg && !hs) {
    reject(6);
    return;
  }
  if (bmg) { // the bitmap's global atomics complete before the component scan reads it
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    wsync();
  }
  // runs -> components: cst[c] / cen[c] per bucket in bucket-index order
  uint32_t *const cst = cg ? hs + 3 * U + (bmg ? Wr : 0) : L.buf + W, *const cen = cst + NR;
  uint32_t ncomp = 0, cbase = 0, NCD = 0;
  for (uint32_t q = 0; q < nbk; q++) {
    const uint32_t wc = rdlane(words, q);
    if (!wc) continue;
    const uint32_t wo = rdlane(woff, q), base = rdlane(dbase, q);
    const uint32_t first_c = NCD;
    for (uint32_t w0 = 0; w0 < wc; w0 += 64) {
      const uint32_t kw = w0 + lane;
      const bool v = kw < wc;
      const uint32_t bits = v ? bmp[wo + kw] : 0;
      const uint32_t prev = (v && kw > 0) ? bmp[wo + kw - 1] >> 31 : 0;
      const uint32_t nxt = (v && kw + 1 < wc) ? bmp[wo + kw + 1] & 1 : 0;
      const uint32_t stb = bits & ~((bits << 1) | prev), enb = bits & ~((bits >> 1) | (nxt << 31));
      const uint32_t ns = (uint32_t)__builtin_popcount(stb);
      const uint32_t inc = wincl(ns, lane), tot = rdlane(inc, 63);
      const uint32_t cb = NCD + inc - ns, clk0 = base + 32 * kw;
      uint32_t x = stb;
      while (x) {
        const uint32_t bpos = (uint32_t)__builtin_ctz(x);
        cst[cb + (uint32_t)__builtin_popcount(stb & ((1u << bpos) - 1))] = clk0 + bpos;
        x &= x - 1;
      }
      x = enb;
      while (x) {
        const uint32_t bpos = (uint32_t)__builtin_ctz(x);
        const uint32_t upto = bpos == 31 ? stb : (stb & ((2u << bpos) - 1));
        cen[cb + (uint32_t)__builtin_popcount(upto) - 1] = clk0 + bpos + 1;
        x &= x - 1;
      }
      NCD += tot;
    }
    if (lane == q) {
      ncomp = NCD - first_c;
      cbase = first_c;
    }
  }
  wsync();
  stamp(5);
  LEAN_STOP(5)
  // component bytes per client
  uint32_t dsb = 0;
  for (uint32_t q = 0; q < nbk; q++) {
    const uint32_t nq = rdlane(ncomp, q), cq = rdlane(cbase, q);
    uint32_t acc = 0;
    for (uint32_t c0 = 0; c0 < nq; c0 += 64) {
      const uint32_t c = cq + c0 + lane;
      const uint32_t sz = c0 + lane < nq ? varlen(cst[c]) + varlen(cen[c] - cst[c]) : 0;
      acc += rdlane(wincl(sz, lane), 63);
    }
    if (lane == q) dsb = acc;
  }
  // client order and entry offsets (the wave, D <= 16); entry offsets [16] at the end of buf
  // (free once the ranges are scattered)
  uint32_t *const eoff = L.buf + LN_BUF - LN_ORD;
  const uint32_t ds_start = blocks_size;
  uint32_t total = 0;
  const uint32_t myeo = lean_ds_order_wave(lane, nbk, hasd, dsf, cl, hasd ? varlen(cl) + varlen(ncomp) + dsb : 0,
                                           ds_start + varlen(D), eoff, total);
  if (lane == 0) {
    Writer wr{out, ds_start};
    w_var(wr, D);
  }
  LEAN_STOP(6)
  if (hasd) {
    Writer wr{out, myeo};
    w_var(wr, cl);
    w_var(wr, ncomp);
  }
  for (uint32_t q = 0; q < nbk; q++) {
    const uint32_t nq = rdlane(ncomp, q), cq = rdlane(cbase, q);
    if (!nq) continue;
    const uint32_t eo = rdlane(myeo, q) + varlen(rdlane(cl, q)) + varlen(nq);
    uint32_t acc = 0;
    for (uint32_t c0 = 0; c0 < nq; c0 += 64) {
      const uint32_t c = cq + c0 + lane;
      const bool v = c0 + lane < nq;
      const uint32_t s0 = v ? cst[c] : 0, ln = v ? cen[c] - s0 : 0;
      const uint32_t sz = v ? varlen(s0) + varlen(ln) : 0;
      const uint32_t inc = wincl(sz, lane);
      if (v) {
        Writer wr{out, eo + acc + inc - sz};
        w_var(wr, s0);
        w_var(wr, ln);
      }
      acc += rdlane(inc, 63);
    }
  }
  if (lane == 0) {
    o.path[d] = 0;
    o.status[d] = 0;
    o.out_len[d] = total;
    o.out_start[d] = slot;
    // batch output bytes: 64 counters 64 B apart (one address for a million documents
    // serialises the L2 atomics: +7 ms on C3)
    if (o.lean_total) atomicAdd(o.lean_total + 8 * (d & 63), (unsigned long long)total);
  }
  stamp(6);
  if (STAMPS && lane == 0) {
    tst[15] = 0x1EA4;
    for (int q = 0; q < 16; q++) o.stamps[(size_t)d * 16 + q] = tst[q];
  }
}

template <int WPB, int OCC, bool STAMPS>
__global__ void __launch_bounds__(64 * WPB, OCC) k_lean(BatchIn b, FastOut o, uint32_t *scr) {
  __shared__ LeanLds lds[WPB];
  ym_set_grammar(b.v1x);
  const uint32_t lane = __lane_id();
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t slot = blockIdx.x * WPB + w;
  if (slot >= b.n_docs) return;
  const uint32_t d = b.order ? __builtin_amdgcn_readfirstlane(b.order[slot]) : slot;
  const uint64_t u0 = b.doc_upd[d], u1 = b.doc_upd[d + 1];
  const uint64_t nb = b.upd_off[u1] - b.upd_off[u0];
  const uint32_t umax = b.lean_umax ? b.lean_umax : LN_UMAX;
  if (scr && (u1 - u0 > LN_AW || nb >= 65536) && u1 - u0 <= umax && nb < (1ull << 31))
    lean_doc<true, STAMPS>(b, o, lds[w], d, lane, scr);
  else
    lean_doc<false, STAMPS>(b, o, lds[w], d, lane, scr);
}

// update-count classes of the dispatch order (longest first)
constexpr uint32_t LN_NCLS = 6;
__device__ __forceinline__ uint32_t lean_class(uint64_t U) {
  return U > 4096 ? 0 : U > 2048 ? 1 : U > 1024 ? 2 : U > 256 ? 3 : U > 64 ? 4 : 5;
}
__global__ void __launch_bounds__(256) k_lean_order_count(const uint64_t *doc_upd, uint32_t n, uint32_t *ctr) {
  __shared__ uint32_t c[LN_NCLS];
  if (threadIdx.x < LN_NCLS) c[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  if (d < n) atomicAdd(&c[lean_class(doc_upd[d + 1] - doc_upd[d])], 1u);
  __syncthreads();
  if (threadIdx.x < LN_NCLS && c[threadIdx.x]) atomicAdd(&ctr[threadIdx.x], c[threadIdx.x]);
}
__global__ void __launch_bounds__(256) k_lean_order_place(const uint64_t *doc_upd, uint32_t n, uint32_t *ctr,
                                                         uint32_t *order) {
  __shared__ uint32_t c[LN_NCLS], base[LN_NCLS];
  if (threadIdx.x < LN_NCLS) c[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t d = blockIdx.x * 256 + threadIdx.x;
  uint32_t k = 0, r = 0;
  if (d < n) {
    k = lean_class(doc_upd[d + 1] - doc_upd[d]);
    r = atomicAdd(&c[k], 1u);
  }
  __syncthreads();
  if (threadIdx.x < LN_NCLS) { // this workgroup's run in its class: class start + claimed offset
    uint32_t start = 0;
    for (uint32_t q = 0; q < threadIdx.x; q++) start += ctr[q];
    base[threadIdx.x] = c[threadIdx.x] ? start + atomicAdd(&ctr[LN_NCLS + threadIdx.x], c[threadIdx.x]) : 0;
  }
  __syncthreads();
  if (d < n) order[base[k] + r] = d;
}
void launch_lean_order(const uint64_t *doc_upd, uint32_t n_docs, uint32_t *ctr, uint32_t *order, hipStream_t s) {
  if (!n_docs) return;
  const dim3 g((n_docs + 255) / 256);
  hipLaunchKernelGGL(k_lean_order_count, g, dim3(256), 0, s, doc_upd, n_docs, ctr);
  hipLaunchKernelGGL(k_lean_order_place, g, dim3(256), 0, s, doc_upd, n_docs, ctr, order);
}

// k_lean's hand-over count (npath[6]) and output bytes (the 64 partials) to the host-mapped
// sig[1..3], then sig[0] = seq; when every document was written it also zeroes the counters
// and partials for the next merge (the host skips its memset).  (Counting finished waves in
// k_lean instead and letting the last one do this took k_lean 0.43 -> 1.03 ms on C2: the
// agent-scope release before each wave's count writes back the XCD's L2.)
__global__ void __launch_bounds__(64) k_lean_fin(uint32_t *counter, uint32_t *sig, uint32_t seq) {
  const uint32_t l = threadIdx.x;
  unsigned long long v = ((const unsigned long long *)(counter + 32))[8 * l];
  uint32_t nrej = counter[32 + 16 * l + 2]; // the hand-over shards (k_lean's reject)
  for (int o = 32; o; o >>= 1) {
    v += __shfl_xor(v, o, 64);
    nrej += __shfl_xor(nrej, o, 64);
  }
  nrej += counter[10];
  __syncthreads(); // every read above precedes the zeroing
  if (nrej == 0)
    for (uint32_t q = l; q < 32 + 64 * 16; q += 64) counter[q] = 0;
  if (l == 0) {
    __hip_atomic_store(sig + 1, nrej, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(sig + 2, (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(sig + 3, (uint32_t)(v >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(sig, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
void launch_lean_fin(uint32_t *counter, uint32_t *sig, uint32_t seq, hipStream_t s) {
  hipLaunchKernelGGL(k_lean_fin, dim3(1), dim3(64), 0, s, counter, sig, seq);
}

void launch_lean(const BatchIn &b, const FastOut &o, uint32_t *scr, hipStream_t s) {
  if (!b.n_docs) return;
  constexpr int WPB = 1;
  // waves per SIMD the register budget is compiled for (LDS allows 6 at 6.8 KB per wave);
  // env YMERGE_LEAN_OCC=4/6 selects the 4- / 6-wave build (A/B)
  static const int occ = getenv("YMERGE_LEAN_OCC") ? atoi(getenv("YMERGE_LEAN_OCC")) : 5;
  const dim3 g((b.n_docs + WPB - 1) / WPB), t(64 * WPB);
  if (o.stamps) {
    if (occ == 4) hipLaunchKernelGGL((k_lean<WPB, 4, true>), g, t, 0, s, b, o, scr);
    else if (occ == 6) hipLaunchKernelGGL((k_lean<WPB, 6, true>), g, t, 0, s, b, o, scr);
    else hipLaunchKernelGGL((k_lean<WPB, 5, true>), g, t, 0, s, b, o, scr);
  } else {
    if (occ == 4) hipLaunchKernelGGL((k_lean<WPB, 4, false>), g, t, 0, s, b, o, scr);
    else if (occ == 6) hipLaunchKernelGGL((k_lean<WPB, 6, false>), g, t, 0, s, b, o, scr);
    else hipLaunchKernelGGL((k_lean<WPB, 5, false>), g, t, 0, s, b, o, scr);
  }
}

} // namespace ym
