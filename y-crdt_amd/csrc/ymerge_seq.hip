// ymerge_seq.hip — exact per-document merge_updates_v1 on gfx950.
//
// k_seq_count: one lane per document validates every update (first error in
//   update order wins, yrs/src/alt.rs:21-25) and sizes the document's scratch.
// k_seq_merge<WRITE>: one lane per document decodes into SoA scratch, runs the
//   yrs merge loop (update.rs:537-704), merges DeleteSets (update.rs:542-548,
//   id_set.rs:385-394) and encodes (update.rs:490-535).  WRITE=false measures the
//   output size, WRITE=true writes at out_off[d].
#include "ycodec.h"
#include "yseq.h"
#include "ywalk.h"
#include "ykernels.h"

namespace ym {

struct CountSink {
  uint32_t NB = 0, NBALL = 0, NE = 0, NR = 0;
  bool unsupported = false;
  YM_INLINE void on_section(uint32_t) {}
  YM_INLINE int on_block(uint32_t, uint32_t, const BlockInfo &bi, uint32_t, uint32_t) {
    NBALL++;
    if (bi.kind != BK_SKIP) NB++;
    if (bi.unsupported) unsupported = true;
    return 0;
  }
  YM_INLINE int on_ds_begin(uint32_t) { return 0; }
  YM_INLINE int on_ds_entry(uint32_t, uint32_t) {
    NE++;
    return 0;
  }
  YM_INLINE void on_ds_range(uint32_t, uint32_t) { NR++; }
  YM_INLINE int on_ds_done() { return 0; }
};

// Documents per wavefront (lpw, 1..64): lane l < lpw of wave w takes document w * lpw + l.  A
// wave's lanes walk different documents and diverge at every step, so a few hundred exact
// documents run one per wavefront (lpw 1: a document's serial walk is the wave's whole time);
// hundreds of thousands run 64 to a wave (ymerge_host.cpp seq_lpw).
__device__ __forceinline__ uint32_t seq_doc(uint32_t lpw, bool &active) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x, lane = g & 63;
  active = lane < lpw;
  return (g >> 6) * lpw + lane;
}

__global__ void __launch_bounds__(64) k_seq_count(BatchIn b, const uint8_t *path, uint8_t *status, uint32_t *counts,
                                                  uint64_t *need_words, uint32_t *n_exact, uint32_t lpw) {
  ym_set_grammar(b.v1x);
  bool active;
  const uint32_t d = seq_doc(lpw, active);
  if (!active || d >= b.n_docs) return;
  if (path && path[d] != 1) {
    need_words[d] = 0;
    return;
  }
  if (path) atomicAdd(n_exact, 1u);
  uint64_t u0 = b.doc_upd[d], u1 = b.doc_upd[d + 1];
  CountSink s;
  int st = 0;
  for (uint64_t u = u0; u < u1 && !st; u++) {
    uint64_t o0 = b.upd_off[u], o1 = b.upd_off[u + 1];
    st = walk_update(b.bytes + o0, (uint32_t)(o1 - o0), s);
  }
  if (!st && s.unsupported) st = E_UNSUPPORTED;
  status[d] = (uint8_t)st;
  uint32_t U = (uint32_t)(u1 - u0);
  counts[4 * d + 0] = U;
  counts[4 * d + 1] = s.NB;
  counts[4 * d + 2] = s.NE;
  counts[4 * d + 3] = s.NR;
  need_words[d] = st ? 0 : ((seq_words(U, s.NB, s.NE, s.NR) + 1) & ~1ull);
}

// ------------------------------------------------------------------ scratch carve
struct SeqMem {
  uint32_t *b_client, *b_clock, *b_len, *b_pos, *b_kind, *b_upd; // [NB]
  uint32_t *upd_beg;                                             // [U+1]
  uint32_t *dec_pos, *heap;                                      // [U]
  int32_t *dec_t;                                                // [U]
  uint32_t *em_blk, *em_off, *em_clock, *em_len, *em_kind, *em_client; // [EM]
  uint32_t *e_client, *e_upd, *e_tpos, *e_live, *e_rbeg, *e_rcnt;      // [NE]
  uint32_t *r_start, *r_end, *r_entry;                                  // [NR]
  uint64_t *k64, *t64;                                                  // [M+1]
  uint32_t *v32, *tv32;                                                 // [M+1]
  uint32_t *hb_keys;                                                    // [NE+1]
  uint32_t *hb_slot, *hb_tmp;                                           // [4NE+64]
  uint32_t hb_cap;
};
__device__ inline SeqMem seq_carve(uint32_t *w, uint32_t U, uint32_t NB, uint32_t NE, uint32_t NR) {
  SeqMem m;
  uint64_t M = NB > NE ? NB : NE;
  if (NR > M) M = NR;
  uint64_t EM = 2ull * NB + 2;
  uint64_t o = 0;
  auto take = [&](uint64_t k) {
    uint32_t *p = w + o;
    o += k;
    return p;
  };
  // 64-bit arrays first (8-byte aligned: scratch base is 8-byte aligned and o even)
  m.k64 = (uint64_t *)take(2 * (M + 1));
  m.t64 = (uint64_t *)take(2 * (M + 1));
  m.v32 = take(M + 1);
  m.tv32 = take(M + 1);
  m.b_client = take(NB);
  m.b_clock = take(NB);
  m.b_len = take(NB);
  m.b_pos = take(NB);
  m.b_kind = take(NB);
  m.b_upd = take(NB);
  m.upd_beg = take(U + 1);
  m.dec_pos = take(U + 1);
  m.heap = take(U + 1);
  m.dec_t = (int32_t *)take(U + 1);
  m.em_blk = take(EM);
  m.em_off = take(EM);
  m.em_clock = take(EM);
  m.em_len = take(EM);
  m.em_kind = take(EM);
  m.em_client = take(EM);
  m.e_client = take(NE);
  m.e_upd = take(NE);
  m.e_tpos = take(NE);
  m.e_live = take(NE);
  m.e_rbeg = take(NE);
  m.e_rcnt = take(NE);
  m.r_start = take(NR);
  m.r_end = take(NR);
  m.r_entry = take(NR);
  m.hb_keys = take(NE + 1);
  m.hb_cap = 4 * NE + 64;
  m.hb_slot = take(m.hb_cap);
  m.hb_tmp = take(m.hb_cap);
  return m;
}

// Per-update table order for updates with more than DS_SMALL DeleteSet entries: the
// same HashMap::insert restatement as ds_small_order, over the document's global
// table scratch (used again only by the later DeleteSet merge).
__device__ __noinline__ void ds_large_order(SeqMem &m, uint32_t ebase, uint32_t n) {
  GHB t{m.hb_slot, m.hb_keys, m.hb_cap, 0, 0, 0};
  uint32_t *pos = m.e_tpos + ebase;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t c = m.e_client[ebase + i];
    pos[i] = 0;
    t.reserve(1, m.hb_tmp); // n <= NE: 4 NE + 64 slots always suffice
    int e = t.find(c);
    if (e >= 0) {
      pos[e] = DS_DEAD;
      for (uint32_t s = 0; s < t.buckets; s++)
        if (t.slot[s] == (uint32_t)e + 1) t.slot[s] = i + 1;
      t.keys[i] = c;
    } else
      t.place(c, i);
  }
  uint32_t k = 0;
  for (uint32_t s = 0; s < t.buckets; s++)
    if (t.slot[s]) pos[t.slot[s] - 1] = k++;
}

struct FillSink {
  SeqMem *m;
  uint32_t upd, nb, ne, nr, ebase;
  const uint8_t *doc_base;
  const uint8_t *upd_base;
  YM_INLINE void on_section(uint32_t) {}
  YM_INLINE int on_block(uint32_t client, uint32_t clock, const BlockInfo &bi, uint32_t bpos, uint32_t) {
    if (bi.kind == BK_SKIP) return 0;
    m->b_client[nb] = client;
    m->b_clock[nb] = clock;
    m->b_len[nb] = bi.len;
    m->b_pos[nb] = (uint32_t)(upd_base - doc_base) + bpos;
    m->b_kind[nb] = bi.kind;
    m->b_upd[nb] = upd;
    nb++;
    return 0;
  }
  YM_INLINE int on_ds_begin(uint32_t) {
    ebase = ne;
    return 0;
  }
  YM_INLINE int on_ds_entry(uint32_t client, uint32_t nrng) {
    m->e_client[ne] = client;
    m->e_upd[ne] = upd;
    m->e_live[ne] = 1;
    m->e_rbeg[ne] = nr;
    m->e_rcnt[ne] = nrng;
    ne++;
    return 0;
  }
  YM_INLINE void on_ds_range(uint32_t s, uint32_t e) {
    m->r_start[nr] = s;
    m->r_end[nr] = e;
    m->r_entry[nr] = ne - 1;
    nr++;
  }
  YM_INLINE int on_ds_done() {
    uint32_t n = ne - ebase;
    if (n == 1) m->e_tpos[ebase] = 0;
    else if (n >= 2) {
      if (n <= DS_SMALL) ds_small_order(m->e_client + ebase, n, m->e_tpos + ebase);
      else ds_large_order(*m, ebase, n);
      for (uint32_t i = 0; i < n; i++)
        if (m->e_tpos[ebase + i] == DS_DEAD) m->e_live[ebase + i] = 0;
    }
    return 0;
  }
};

struct Car {
  uint32_t blk, off, client, clock, len, kind;
};

// BlockCarrier::splice (update.rs:795-816; block.rs:435-478, 1837-1879)
__device__ int car_splice(const uint8_t *doc, uint32_t doc_len, const SeqMem &m, const Car &c, uint32_t diff,
                          Car &out) {
  out = c;
  out.clock = c.clock + diff;
  out.off = c.off + diff;
  if (c.kind != BK_ITEM) {
    out.len = c.len - diff;
    return 0;
  }
  // locate content of the original item
  Cur q{doc, doc_len, m.b_pos[c.blk]};
  uint8_t info;
  bool cn;
  uint32_t v;
  rd_u8(q, info);
  if (info & 0x80) {
    rd_var_u32(q, v, cn);
    rd_var_u32(q, v, cn);
  }
  if (info & 0x40) {
    rd_var_u32(q, v, cn);
    rd_var_u32(q, v, cn);
  }
  if ((info & 0xC0) == 0) {
    uint32_t pi;
    rd_var_u32(q, pi, cn);
    if (pi == 1) {
      rd_var_u32(q, v, cn);
      q.i += v;
    } else {
      rd_var_u32(q, v, cn);
      rd_var_u32(q, v, cn);
    }
    if (info & 0x20) {
      rd_var_u32(q, v, cn);
      q.i += v;
    }
  }
  uint32_t olen = m.b_len[c.blk];
  switch (info & 15) {
  case 1: case 2: case 8:
    if (diff > olen) return E_PANIC;
    out.len = olen - diff;
    return 0;
  case 4: {
    rd_var_u32(q, v, cn);
    uint32_t bo;
    YM_TRY(str_split16(doc + q.i, v, diff, bo));
    out.len = str_len16(doc + q.i + bo, v - bo);
    return 0;
  }
  default: return E_PANIC; // ItemContent::splice -> None; .unwrap()
  }
}

struct SeqCtx {
  const uint8_t *doc;
  uint32_t doc_len;
  SeqMem m;
  uint32_t U, NB, NE, NR, nem;
};

__device__ __forceinline__ bool cur_of(const SeqCtx &x, uint32_t u, Car &c) {
  uint32_t p = x.m.dec_pos[u];
  if (p >= x.m.upd_beg[u + 1]) return false;
  c.blk = p;
  c.off = 0;
  c.client = x.m.b_client[p];
  c.clock = x.m.b_clock[p];
  c.len = x.m.b_len[p];
  c.kind = x.m.b_kind[p];
  return true;
}
__device__ __forceinline__ bool has_cur(const SeqCtx &x, uint32_t u) { return x.m.dec_pos[u] < x.m.upd_beg[u + 1]; }
// heap order: client desc, clock asc, last re-insert desc, input index asc
__device__ __forceinline__ bool heap_less(const SeqCtx &x, uint32_t a, uint32_t b) {
  uint32_t pa = x.m.dec_pos[a], pb = x.m.dec_pos[b];
  uint32_t ca = x.m.b_client[pa], cb = x.m.b_client[pb];
  if (ca != cb) return ca > cb;
  uint32_t ka = x.m.b_clock[pa], kb = x.m.b_clock[pb];
  if (ka != kb) return ka < kb;
  int32_t ta = x.m.dec_t[a], tb = x.m.dec_t[b];
  if (ta != tb) return ta > tb;
  return a < b;
}
// yrs comparator (update.rs:572-589) as is_less; `small` = Rust's insertion-sort regime
// (<= SORT_SMALL live decoders).  Above it the Item/GC tie reads as Equal.
constexpr uint32_t SORT_SMALL = 20;
__device__ __forceinline__ bool dec_less(const SeqCtx &x, uint32_t a, uint32_t b, bool small) {
  uint32_t pa = x.m.dec_pos[a], pb = x.m.dec_pos[b];
  uint32_t ca = x.m.b_client[pa], cb = x.m.b_client[pb];
  if (ca != cb) return ca > cb;
  uint32_t ka = x.m.b_clock[pa], kb = x.m.b_clock[pb];
  if (ka == kb) return small && x.m.b_kind[pa] != x.m.b_kind[pb];
  return ka < kb;
}
__device__ void heap_push(SeqCtx &x, uint32_t &nh, uint32_t d) {
  uint32_t *h = x.m.heap;
  uint32_t i = nh++;
  h[i] = d;
  while (i > 0) {
    uint32_t p = (i - 1) / 2;
    if (!heap_less(x, h[i], h[p])) break;
    uint32_t t = h[i];
    h[i] = h[p];
    h[p] = t;
    i = p;
  }
}
__device__ uint32_t heap_pop(SeqCtx &x, uint32_t &nh) {
  uint32_t *h = x.m.heap;
  uint32_t top = h[0];
  h[0] = h[--nh];
  uint32_t i = 0;
  for (;;) {
    uint32_t l = 2 * i + 1, r = l + 1, mm = i;
    if (l < nh && heap_less(x, h[l], h[mm])) mm = l;
    if (r < nh && heap_less(x, h[r], h[mm])) mm = r;
    if (mm == i) break;
    uint32_t t = h[i];
    h[i] = h[mm];
    h[mm] = t;
    i = mm;
  }
  return top;
}

__device__ int seq_merge_blocks(SeqCtx &x) {
  SeqMem &m = x.m;
  // Sort policy (oracle merge_blocks): a heap in the regime the comparator is consistent
  // (> SORT_SMALL live decoders, or no Item/GC tie at one (client, clock) anywhere); the
  // literal insertion-sort loop once <= SORT_SMALL are live and such a tie exists.
  for (uint32_t i = 0; i < x.NB; i++) {
    m.k64[i] = ((uint64_t)m.b_client[i] << 32) | m.b_clock[i];
    m.v32[i] = m.b_kind[i];
  }
  seq_sort64(m.k64, m.v32, m.t64, m.tv32, x.NB);
  bool anomaly = false;
  for (uint32_t i = 1; i < x.NB; i++)
    if (m.k64[i] == m.k64[i - 1] && m.v32[i] != m.v32[i - 1]) anomaly = true;

  uint32_t na = 0, nh = 0;
  for (uint32_t u = 0; u < x.U; u++) {
    m.dec_pos[u] = m.upd_beg[u];
    m.dec_t[u] = -1;
    if (has_cur(x, u)) na++;
  }
  bool literal = anomaly && na <= SORT_SMALL;
  na = 0;
  for (uint32_t u = 0; u < x.U; u++) {
    if (!has_cur(x, u)) continue;
    if (literal)
      m.heap[na++] = u; // heap[] doubles as the decoder array
    else
      heap_push(x, nh, u);
  }
  uint32_t last = ~0u;
  x.nem = 0;
  auto emit = [&](const Car &c) {
    uint32_t k = x.nem++;
    m.em_blk[k] = c.blk;
    m.em_off[k] = c.off;
    m.em_clock[k] = c.clock;
    m.em_len[k] = c.len;
    m.em_kind[k] = c.kind;
    m.em_client[k] = c.client;
  };
  Car cw{};
  bool has_cw = false;
  for (int32_t iter = 0;; iter++) {
    uint32_t d;
    if (!literal && anomaly && nh <= SORT_SMALL) { // deque = [popped last] + heap order
      uint32_t tmp[SORT_SMALL], nt = 0;
      while (nh) {
        uint32_t e = heap_pop(x, nh);
        if (e != last) tmp[nt++] = e;
      }
      na = 0;
      if (last != ~0u && has_cur(x, last)) m.heap[na++] = last;
      for (uint32_t i = 0; i < nt; i++) m.heap[na++] = tmp[i];
      literal = true;
    }
    if (literal) {
      uint32_t k = 0;
      for (uint32_t i = 0; i < na; i++)
        if (has_cur(x, m.heap[i])) m.heap[k++] = m.heap[i];
      na = k;
      bool small = na <= SORT_SMALL;
      for (uint32_t i = 1; i < na; i++) { // insertion_sort_shift_left
        uint32_t tmp = m.heap[i], j = i;
        while (j > 0 && dec_less(x, tmp, m.heap[j - 1], small)) {
          m.heap[j] = m.heap[j - 1];
          j--;
        }
        m.heap[j] = tmp;
      }
      if (na == 0) break;
      d = m.heap[0];
    } else {
      if (nh == 0) break;
      d = heap_pop(x, nh);
    }
    last = d;
    Car b;
    cur_of(x, d, b);
    uint32_t first_client = b.client;
    if (has_cw) {
      bool iterated = false;
      uint32_t cwl = cw.clock + cw.len;
      while (cur_of(x, d, b) && (uint32_t)(b.clock + b.len) <= cwl && b.client >= cw.client) {
        m.dec_pos[d]++;
        iterated = true;
      }
      if (!cur_of(x, d, b)) goto next;
      if (b.client != first_client || (iterated && b.clock > cwl)) goto next;
      if (first_client != cw.client) {
        emit(cw);
        cw = b;
        m.dec_pos[d]++;
      } else if (cwl < b.clock) {
        if (cw.kind == BK_SKIP) {
          cw.len = b.clock + b.len - cw.clock;
        } else {
          emit(cw);
          cw = Car{~0u, 0, first_client, cwl, b.clock - cwl, BK_SKIP};
        }
      } else {
        uint32_t diff = cwl > b.clock ? cwl - b.clock : 0;
        Car slice;
        bool has_slice = false;
        if (diff > 0) {
          if (cw.kind == BK_SKIP) {
            cw.len -= diff;
          } else {
            YM_TRY(car_splice(x.doc, x.doc_len, m, b, diff, slice));
            has_slice = true;
          }
        }
        Car cur = has_slice ? slice : b;
        if (cw.kind == BK_SKIP && cur.kind == BK_SKIP) {
          cw.len += cur.len;
        } else {
          emit(cw);
          cw = cur;
          m.dec_pos[d]++;
        }
      }
    } else {
      cw = b;
      has_cw = true;
      m.dec_pos[d]++;
    }
    while (cur_of(x, d, b)) {
      if (b.client == first_client && b.clock == (uint32_t)(cw.clock + cw.len)) {
        emit(cw);
        cw = b;
        m.dec_pos[d]++;
      } else
        break;
    }
  next:
    if (!literal && has_cur(x, d)) {
      m.dec_t[d] = iter;
      heap_push(x, nh, d);
    }
  }
  if (has_cw) emit(cw);
  return 0;
}

// encode_diff with an empty state vector over emitted carriers (update.rs:490-535)
template <class W> __device__ int seq_encode_blocks(SeqCtx &x, W &w) {
  SeqMem &m = x.m;
  // pass 1: number of clients with a selectable first block
  uint32_t ncl = 0;
  for (uint32_t i = 0; i < x.nem;) {
    uint32_t j = i;
    bool sel = false;
    while (j < x.nem && m.em_client[j] == m.em_client[i]) {
      if (!sel && m.em_kind[j] != BK_SKIP && (uint32_t)(m.em_clock[j] + m.em_len[j]) > 0) sel = true;
      j++;
    }
    ncl += sel;
    i = j;
  }
  w_var(w, ncl);
  for (uint32_t i = 0; i < x.nem;) {
    uint32_t j = i, first = ~0u;
    while (j < x.nem && m.em_client[j] == m.em_client[i]) {
      if (first == ~0u && m.em_kind[j] != BK_SKIP && (uint32_t)(m.em_clock[j] + m.em_len[j]) > 0) first = j;
      j++;
    }
    if (first != ~0u) {
      w_var(w, j - first);
      w_var(w, m.em_client[i]);
      w_var(w, m.em_clock[first]);
      for (uint32_t k = first; k < j; k++) {
        uint32_t kind = m.em_kind[k];
        if (kind == BK_SKIP || kind == BK_GC) {
          w.u8(kind == BK_SKIP ? 10 : 0);
          w_var(w, m.em_len[k]);
        } else {
          uint32_t bi = m.em_blk[k];
          YM_TRY(emit_block(x.doc, x.doc_len, m.b_pos[bi], m.b_client[bi], m.b_clock[bi], m.b_len[bi], m.em_off[k], w));
        }
      }
    }
    i = j;
  }
  return 0;
}

// DeleteSet union in yrs' table order (update.rs:542-548, id_set.rs:129-164, 385-410)
template <class W> __device__ int seq_encode_ds(SeqCtx &x, W &w) {
  SeqMem &m = x.m;
  GHB t{m.hb_slot, m.hb_keys, m.hb_cap, 0, 0, 0};
  for (uint32_t i = 0; i < x.NE;) { // entries grouped by update, stream order
    uint32_t j = i;
    while (j < x.NE && m.e_upd[j] == m.e_upd[i]) j++;
    uint32_t nlive = 0;
    for (uint32_t k = i; k < j; k++) nlive += m.e_live[k];
    for (uint32_t tp = 0; tp < nlive; tp++) {
      for (uint32_t k = i; k < j; k++) {
        if (!m.e_live[k] || m.e_tpos[k] != tp) continue;
        uint32_t c = m.e_client[k];
        if (t.find(c) < 0) {
          if (!t.reserve(1, m.hb_tmp)) return E_UNSUPPORTED;
          t.place(c, t.items);
        }
      }
    }
    i = j;
  }
  // live ranges sorted by (client, start)
  uint32_t n = 0;
  for (uint32_t r = 0; r < x.NR; r++) {
    if (!m.e_live[m.r_entry[r]]) continue;
    m.k64[n] = ((uint64_t)m.e_client[m.r_entry[r]] << 32) | m.r_start[r];
    m.v32[n] = r;
    n++;
  }
  seq_sort64(m.k64, m.v32, m.t64, m.tv32, n);
  w_var(w, t.items);
  for (uint32_t s = 0; s < t.buckets; s++) {
    if (!t.slot[s]) continue;
    uint32_t client = t.keys[t.slot[s] - 1];
    // lower bound of client in k64
    uint32_t lo = 0, hi = n;
    uint64_t key = (uint64_t)client << 32;
    while (lo < hi) {
      uint32_t mid = (lo + hi) / 2;
      if (m.k64[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    uint32_t a = lo, bnd = lo;
    while (bnd < n && (uint32_t)(m.k64[bnd] >> 32) == client) bnd++;
    uint32_t ncomp = 0;
    for (uint32_t k = a; k < bnd;) {
      uint32_t e = m.r_end[m.v32[k]];
      uint32_t q = k + 1;
      while (q < bnd && m.r_start[m.v32[q]] <= e) {
        uint32_t e2 = m.r_end[m.v32[q]];
        if (e2 > e) e = e2;
        q++;
      }
      ncomp++;
      k = q;
    }
    w_var(w, client);
    w_var(w, ncomp);
    for (uint32_t k = a; k < bnd;) {
      uint32_t s0 = m.r_start[m.v32[k]], e = m.r_end[m.v32[k]];
      uint32_t q = k + 1;
      while (q < bnd && m.r_start[m.v32[q]] <= e) {
        uint32_t e2 = m.r_end[m.v32[q]];
        if (e2 > e) e = e2;
        q++;
      }
      w_var(w, s0);
      w_var(w, e - s0);
      k = q;
    }
  }
  return 0;
}

__device__ int seq_fill(SeqCtx &x, const BatchIn &b, uint64_t u0) {
  FillSink s;
  s.m = &x.m;
  s.nb = s.ne = s.nr = 0;
  s.doc_base = x.doc;
  for (uint32_t u = 0; u < x.U; u++) {
    uint64_t o0 = b.upd_off[u0 + u], o1 = b.upd_off[u0 + u + 1];
    s.upd = u;
    s.upd_base = b.bytes + o0;
    x.m.upd_beg[u] = s.nb;
    uint32_t nb0 = s.nb;
    YM_TRY(walk_update(b.bytes + o0, (uint32_t)(o1 - o0), s));
    // IntoBlocks: this update's blocks ordered client desc (stable)
    for (uint32_t i = nb0 + 1; i < s.nb; i++) {
      uint32_t j = i;
      while (j > nb0 && x.m.b_client[j - 1] < x.m.b_client[j]) {
        uint32_t *arrs[6] = {x.m.b_client, x.m.b_clock, x.m.b_len, x.m.b_pos, x.m.b_kind, x.m.b_upd};
        for (int a = 0; a < 6; a++) {
          uint32_t t = arrs[a][j];
          arrs[a][j] = arrs[a][j - 1];
          arrs[a][j - 1] = t;
        }
        j--;
      }
    }
  }
  x.m.upd_beg[x.U] = s.nb;
  return 0;
}

template <bool WRITE>
__global__ void __launch_bounds__(64) k_seq_merge(BatchIn b, const uint8_t *path, const uint8_t *status,
                                                  const uint32_t *counts, const uint64_t *scr_off, uint32_t *scratch,
                                                  uint64_t *sizes, const uint64_t *out_off, uint8_t *out,
                                                  uint64_t out_base, uint64_t *out_start, uint64_t *out_len,
                                                  uint8_t *status_out, uint32_t lpw, uint64_t *dbg) {
  ym_set_grammar(b.v1x);
  bool active;
  const uint32_t d = seq_doc(lpw, active);
  if (!active || d >= b.n_docs) return;
  const uint64_t t0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
  if (path && path[d] != 1) {
    if (!WRITE) sizes[d] = 0;
    return;
  }
  if (status[d]) {
    if (!WRITE) sizes[d] = 0;
    if (WRITE && out_len) {
      out_len[d] = 0;
      out_start[d] = out_base + out_off[d];
    }
    return;
  }
  SeqCtx x;
  x.U = counts[4 * d + 0];
  x.NB = counts[4 * d + 1];
  x.NE = counts[4 * d + 2];
  x.NR = counts[4 * d + 3];
  uint64_t u0 = b.doc_upd[d];
  uint64_t dstart = b.upd_off[u0], dend = b.upd_off[b.doc_upd[d + 1]];
  x.doc = b.bytes + dstart;
  x.doc_len = (uint32_t)(dend - dstart);
  x.m = seq_carve(scratch + scr_off[d], x.U, x.NB, x.NE, x.NR);
  int err = seq_fill(x, b, u0);
  if (!err) err = seq_merge_blocks(x);
  if (WRITE) {
    Writer w{out + out_base + out_off[d], 0};
    if (!err) err = seq_encode_blocks(x, w);
    if (!err) err = seq_encode_ds(x, w);
    if (out_len) {
      out_start[d] = out_base + out_off[d];
      out_len[d] = w.n;
    }
    if (dbg) dbg[d] = __builtin_amdgcn_s_memtime() - t0; // diagnostic (env YMERGE_SEQ_DBG): cycles
  } else {
    Counter c;
    if (!err) err = seq_encode_blocks(x, c);
    if (!err) err = seq_encode_ds(x, c);
    sizes[d] = err ? 0 : c.n;
    if (err) status_out[d] = (uint8_t)err;
  }
}

} // namespace ym

// ------------------------------------------------------------------ launchers
namespace ym {
void launch_seq_count(const BatchIn &b, const uint8_t *path, uint8_t *status, uint32_t *counts, uint64_t *need,
                      uint32_t *n_exact, hipStream_t s, uint32_t lpw) {
  const uint32_t nb = (uint32_t)((b.n_docs + lpw - 1) / lpw); // one wavefront per workgroup
  if (nb) hipLaunchKernelGGL(k_seq_count, dim3(nb), dim3(64), 0, s, b, path, status, counts, need, n_exact, lpw);
}
void launch_seq_merge(bool write, const BatchIn &b, const uint8_t *path, const uint8_t *status, const uint32_t *counts,
                      const uint64_t *scr_off, uint32_t *scratch, uint64_t *sizes, const uint64_t *out_off,
                      uint8_t *out, uint64_t out_base, uint64_t *out_start, uint64_t *out_len, uint8_t *status_out,
                      hipStream_t s, uint32_t lpw, uint64_t *dbg) {
  const uint32_t nb = (uint32_t)((b.n_docs + lpw - 1) / lpw);
  if (!nb) return;
  if (write)
    hipLaunchKernelGGL(k_seq_merge<true>, dim3(nb), dim3(64), 0, s, b, path, status, counts, scr_off, scratch, sizes,
                       out_off, out, out_base, out_start, out_len, status_out, lpw, dbg);
  else
    hipLaunchKernelGGL(k_seq_merge<false>, dim3(nb), dim3(64), 0, s, b, path, status, counts, scr_off, scratch,
                       sizes, out_off, out, out_base, out_start, out_len, status_out, lpw, dbg);
}
} // namespace ym
