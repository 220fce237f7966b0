// ywalk.h — one pass over a v1 update (Decode for Update, yrs/src/update.rs:714-749
// + DeleteSet::decode, id_set.rs:412-426) driving a sink; shared by every kernel.
#pragma once
#include "ycodec.h"

namespace ym {

// ------------------------------------------------------------------ update walk
// Sink interface: on_section, on_block, on_ds_entry, on_ds_range, on_ds_done.
struct TrackClients {
  uint32_t client[8], count[8];
  uint32_t n;
  YM_INLINE void reset() { n = 0; }
  // returns blocks already recorded for `client` in this update (exact for <= 8 clients)
  YM_INLINE uint32_t *slot(uint32_t c) {
    for (uint32_t i = 0; i < n; i++)
      if (client[i] == c) return &count[i];
    if (n < 8) {
      client[n] = c;
      count[n] = 0;
      return &count[n++];
    }
    return nullptr;
  }
};

template <class S> YM_INLINE int walk_update(const uint8_t *p, uint32_t n, S &s) {
  Cur c{p, n, 0};
  bool cn;
  uint32_t ncl;
  YM_TRY(rd_var_u32(c, ncl, cn));
  if (ncl && cap_to_buckets(ncl) * 41ull > ALLOC_LIMIT) return E_NEM; // try_reserve, (u64, VecDeque) = 40 B
  TrackClients tc;
  tc.reset();
  for (uint32_t i = 0; i < ncl; i++) {
    uint32_t nb, client, clock;
    YM_TRY(rd_var_u32(c, nb, cn));
    YM_TRY(rd_var_u32(c, client, cn));
    YM_TRY(rd_var_u32(c, clock, cn));
    uint32_t *cnt = ncl > 1 ? tc.slot(client) : nullptr;
    uint64_t existing = cnt ? *cnt : 0;
    if ((existing + nb) * 32ull > ALLOC_LIMIT) return E_NEM; // VecDeque<BlockCarrier>::try_reserve
    s.on_section(client);
    for (uint32_t j = 0; j < nb; j++) {
      uint32_t bpos = c.i;
      BlockInfo bi;
      YM_TRY(parse_block(c, bi));
      if (bi.kind == BK_ITEM && bi.len == 0) continue; // Item::new -> None
      if ((uint64_t)clock + bi.len > 0xFFFFFFFFull) return E_PANIC;
      YM_TRY(s.on_block(client, clock, bi, bpos, c.i - bpos));
      if (cnt) (*cnt)++;
      clock += bi.len;
    }
  }
  uint32_t nds;
  YM_TRY(rd_var_u32(c, nds, cn));
  YM_TRY(s.on_ds_begin(nds));
  for (uint32_t i = 0; i < nds; i++) {
    uint32_t client, nr;
    YM_TRY(rd_var_u32(c, client, cn));
    YM_TRY(rd_var_u32(c, nr, cn));
    YM_TRY(s.on_ds_entry(client, nr));
    for (uint32_t k = 0; k < nr; k++) {
      uint32_t st, ln;
      YM_TRY(rd_var_u32(c, st, cn));
      YM_TRY(rd_var_u32(c, ln, cn));
      if ((uint64_t)st + ln > 0xFFFFFFFFull) return E_PANIC;
      s.on_ds_range(st, st + ln);
    }
  }
  return s.on_ds_done();
}

// DS table order of one update: HashMap::insert per entry in stream order
// Per-update DeleteSet table order.  IdSet decoding inserts every (client, ranges)
// entry of one update into a std HashMap (id_set.rs:411-426, HashMap::insert:
// reserve(1), replace in place on a repeated client); the DeleteSet merge later
// iterates that table (update.rs:542-548).  ds_small_order restates the table for
// one update with at most DS_SMALL entries (16 buckets suffice) and reports, per
// entry in stream order, its iteration position or DS_DEAD if a later entry with
// the same client replaced it.  Cold path: single-entry updates never call it.
constexpr uint32_t DS_SMALL = 14;
constexpr uint32_t DS_DEAD = 0xFFFFFFFFu;
__device__ __noinline__ void ds_small_order(const uint32_t *clients, uint32_t n, uint32_t *pos_out) {
  SmallHB<16> hb;
  hb.init_empty();
  for (uint32_t i = 0; i < n; i++) {
    uint32_t c = clients[i];
    pos_out[i] = 0;
    bool existed;
    int e = hb.insert(c, i, existed);
    if (existed) {
      pos_out[e] = DS_DEAD;
      for (uint32_t s = 0; s < hb.buckets; s++)
        if (hb.slot[s] == e + 1) hb.slot[s] = (uint16_t)(i + 1);
      hb.keys[i] = c;
    }
  }
  uint32_t k = 0;
  for (uint32_t s = 0; s < hb.buckets; s++)
    if (hb.slot[s]) pos_out[hb.slot[s] - 1] = k++;
}

// ds_small_order without a stack: for n <= DS_SMALL entries the table has at most 16
// buckets (4 -> 8 -> 16), where hashbrown's group probe (16 control bytes, trailing
// mirror / EMPTY bytes) reduces to linear probing with wrap-around from client & mask.
// Slot -> entry+1 lives in one u64 (4 bits per slot).  Writes every entry's code
// (0x80000000 | iteration position, or 0 if a later entry replaced it) | tag into et.
YM_INLINE uint32_t hb_probe(uint64_t m, uint32_t nb, uint32_t key) {
  uint32_t s = key & (nb - 1);
  while ((m >> (4 * s)) & 15) s = (s + 1) & (nb - 1);
  return s;
}
YM_INLINE void ds_order_packed(const uint32_t *cl, uint32_t n, uint32_t *et, uint32_t tag) {
  uint64_t map = 0;
  uint32_t buckets = 0, items = 0, growth = 0, dead = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t c = cl[i];
    if (growth == 0) { // HashMap::insert -> reserve(1) -> resize (old slots re-placed in slot order)
      const uint32_t full = buckets ? (uint32_t)mask_to_cap(buckets - 1) : 0;
      const uint32_t need = items + 1;
      const uint32_t nb = (uint32_t)cap_to_buckets(need > full + 1 ? need : full + 1);
      uint64_t nm = 0;
      for (uint32_t s = 0; s < buckets; s++) {
        const uint32_t en = (uint32_t)(map >> (4 * s)) & 15;
        if (en) nm |= (uint64_t)en << (4 * hb_probe(nm, nb, cl[en - 1]));
      }
      map = nm;
      buckets = nb;
      growth = (uint32_t)mask_to_cap(nb - 1) - items;
    }
    int fs = -1;
    for (uint32_t s = 0; s < buckets; s++) {
      const uint32_t en = (uint32_t)(map >> (4 * s)) & 15;
      if (en && cl[en - 1] == c) fs = (int)s;
    }
    if (fs >= 0) { // replace in place: the earlier entry is dead
      dead |= 1u << (((uint32_t)(map >> (4 * fs)) & 15) - 1);
      map = (map & ~(15ull << (4 * fs))) | ((uint64_t)(i + 1) << (4 * fs));
    } else {
      map |= (uint64_t)(i + 1) << (4 * hb_probe(map, buckets, c));
      items++;
      growth--;
    }
  }
  uint32_t k = 0;
  for (uint32_t s = 0; s < buckets; s++) {
    const uint32_t en = (uint32_t)(map >> (4 * s)) & 15;
    if (en) et[en - 1] = 0x80000000u | k++ | tag;
  }
  for (uint32_t i = 0; i < n; i++)
    if ((dead >> i) & 1) et[i] = tag;
}

} // namespace ym
