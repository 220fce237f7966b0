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
  __device__ void reset() { n = 0; }
  // returns blocks already recorded for `client` in this update (exact for <= 8 clients)
  __device__ uint32_t *slot(uint32_t c) {
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

template <class S> __device__ int walk_update(const uint8_t *p, uint32_t n, S &s) {
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
    uint32_t *cnt = tc.slot(client);
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
struct DsOrder {
  SmallHB<64> hb;
  uint32_t n;
  __device__ void begin() {
    hb.init_empty();
    n = 0;
  }
  // returns local index of a replaced (now dead) entry, ~0u if none; <0 error
  __device__ int insert(uint32_t client, uint32_t &dead) {
    if (n >= 64) return E_UNSUPPORTED; // device limit: <= 64 DeleteSet entries per update
    bool existed;
    int e = hb.insert(client, n, existed);
    if (e == -2) return E_UNSUPPORTED;
    dead = ~0u;
    if (existed) {
      dead = (uint32_t)e;
      for (uint32_t i = 0; i < hb.buckets; i++)
        if (hb.slot[i] == e + 1) hb.slot[i] = (uint16_t)(n + 1);
      hb.keys[n] = client;
    }
    n++;
    return 0;
  }
};

} // namespace ym
