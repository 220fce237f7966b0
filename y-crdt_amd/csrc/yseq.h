// yseq.h — exact per-document engine (device).  One lane owns one document and
// runs the yrs merge loop (yrs/src/update.rs:537-704) with the decoder ordering
// kept in a binary heap: equivalent to yrs' per-iteration stable sort whenever the
// comparator is consistent; when an Item and a GC start at the same (client,
// clock) the comparator is not (update.rs:580-582) and the lane falls back to a
// literal insertion sort each iteration (Rust's sort for <= 20 elements).
// This path is exact for every document; the parallel LDS path (ydoc_lds.h)
// handles the documents that meet the fast-path precondition.
#pragma once
#include "ycodec.h"

namespace ym {

// per-document scratch (u32 words), carved by layout_words()
struct SeqCounts {
  uint32_t U, NB, NE, NR, NBALL;
};
__device__ __host__ inline uint64_t seq_words(uint32_t U, uint32_t NB, uint32_t NE, uint32_t NR) {
  uint64_t M = (uint64_t)(NB > NE ? NB : NE);
  if (NR > M) M = NR;
  uint64_t EM = 2ull * NB + 2;
  return 6ull * NB + 4ull * (U + 1) + 6ull * EM + 6ull * NE + 3ull * NR + 6ull * (M + 1) + 4ull * (NE + 1) +
         2ull * (4 * NE + 64) + 64;
}

// global-memory SwissTable emulation for one table (slots hold entry+1)
struct GHB {
  uint32_t *slot;
  uint32_t *keys;
  uint32_t cap_slots; // allocated slot capacity
  uint32_t buckets, items, growth_left;
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
    if (!buckets) return -1;
    uint32_t mask = buckets - 1, pos = key & mask, stride = 0;
    for (;;) {
      bool any_empty = false;
      for (uint32_t j = 0; j < 16; j++) {
        uint32_t idx = pos + j;
        if (ctrl_empty(idx)) {
          any_empty = true;
          continue;
        }
        uint32_t s = slot[idx & mask];
        if (s && keys[s - 1] == key) return (int)(s - 1);
      }
      if (any_empty) return -1;
      stride += 16;
      pos = (pos + stride) & mask;
    }
  }
  __device__ bool resize(uint64_t cap, uint32_t *tmp) {
    uint64_t nb = cap_to_buckets(cap);
    if (nb > cap_slots) return false;
    uint32_t ob = buckets;
    for (uint32_t i = 0; i < ob; i++) tmp[i] = slot[i];
    buckets = (uint32_t)nb;
    for (uint32_t i = 0; i < buckets; i++) slot[i] = 0;
    for (uint32_t i = 0; i < ob; i++)
      if (tmp[i]) slot[find_insert_slot(keys[tmp[i] - 1])] = tmp[i];
    growth_left = (uint32_t)mask_to_cap(buckets - 1) - items;
    return true;
  }
  __device__ bool reserve(uint64_t add, uint32_t *tmp) {
    if (add <= growth_left) return true;
    uint64_t full_cap = buckets ? mask_to_cap(buckets - 1) : 0;
    uint64_t need = items + add;
    return resize(need > full_cap + 1 ? need : full_cap + 1, tmp);
  }
  __device__ void place(uint32_t key, uint32_t e) {
    keys[e] = key;
    slot[find_insert_slot(key)] = e + 1;
    items++;
    growth_left--;
  }
};

// bottom-up merge sort of (key, val) by key (stable), single lane
__device__ inline void seq_sort64(uint64_t *k, uint32_t *v, uint64_t *tk, uint32_t *tv, uint32_t n) {
  // insertion sort when already nearly sorted / tiny
  bool sorted = true;
  for (uint32_t i = 1; i < n && sorted; i++) sorted = k[i - 1] <= k[i];
  if (sorted) return;
  for (uint32_t w = 1; w < n; w *= 2) {
    for (uint32_t lo = 0; lo < n; lo += 2 * w) {
      uint32_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
      uint32_t i = lo, j = mid, o = lo;
      while (i < mid && j < hi) {
        if (k[j] < k[i]) {
          tk[o] = k[j];
          tv[o++] = v[j++];
        } else {
          tk[o] = k[i];
          tv[o++] = v[i++];
        }
      }
      while (i < mid) {
        tk[o] = k[i];
        tv[o++] = v[i++];
      }
      while (j < hi) {
        tk[o] = k[j];
        tv[o++] = v[j++];
      }
    }
    for (uint32_t i = 0; i < n; i++) {
      k[i] = tk[i];
      v[i] = tv[i];
    }
  }
}

} // namespace ym
