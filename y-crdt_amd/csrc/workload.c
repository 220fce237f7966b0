/*
 * workload.c — synthetic Yjs v1 update logs for the BASELINE.json configs.
 *
 * A small YATA-shaped text model (runs of (client, clock, len, deleted)) that
 * emits exactly what a Yjs/yrs replica sends per transaction:
 *   insert -> [1][1][client][clock][info][origin][right origin | parent][string][DS 0]
 *             (update.rs:714-749 grammar; origin = last visible char before the
 *              cursor, right origin = the next item in list order, as Yjs'
 *              findPosition leaves them)
 *   delete -> [0][DS: nClients (client nRanges (clock len)*)*]   (id_set.rs:401-426)
 * Nothing here integrates or merges: the engine under test does that.
 *
 * Configs (BASELINE.json):
 *   C1  replay of an editing trace (automerge-paper), one client, one update per txn
 *   C2  n docs x k ops, 1-4 clients, 80/20 insert/delete, replicas synced after each op
 *   C3  Zipf(1.5)-sized op counts on [1, 10^4]
 *   C4  delete-heavy docs: a GC'd snapshot + the per-op log with 10% withheld and
 *       5% stale duplicates (partial overlaps -> exact path)
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint32_t cl, clock, len;
  uint8_t del;
} run_t;
typedef struct {
  uint8_t *d;
  size_t n, cap;
} bytes_t;
static void put(bytes_t *b, uint8_t x) {
  if (b->n == b->cap) {
    b->cap = b->cap ? b->cap * 2 : 256;
    b->d = realloc(b->d, b->cap);
  }
  b->d[b->n++] = x;
}
static void putv(bytes_t *b, uint64_t v) {
  while (v >= 0x80) {
    put(b, (uint8_t)(v | 0x80));
    v >>= 7;
  }
  put(b, (uint8_t)v);
}
static void putbytes(bytes_t *b, const uint8_t *s, size_t n) {
  for (size_t i = 0; i < n; i++) put(b, s[i]);
}

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static uint32_t urand(uint64_t *s, uint32_t n) { return (uint32_t)(splitmix64(s) % n); }

typedef struct {
  run_t *r;
  size_t n, cap;
  uint64_t visible;
  uint32_t *client_ids, *clocks;
  uint32_t n_clients;
} doc_t;

static void runs_insert_at(doc_t *d, size_t i, run_t x) {
  if (d->n == d->cap) {
    d->cap = d->cap ? d->cap * 2 : 64;
    d->r = realloc(d->r, d->cap * sizeof(run_t));
  }
  memmove(d->r + i + 1, d->r + i, (d->n - i) * sizeof(run_t));
  d->r[i] = x;
  d->n++;
}
/* split run i so that it ends after `o` chars; returns nothing */
static void runs_split(doc_t *d, size_t i, uint32_t o) {
  run_t a = d->r[i], b = a;
  a.len = o;
  b.clock += o;
  b.len -= o;
  d->r[i] = a;
  runs_insert_at(d, i + 1, b);
}

/* Yjs-style insert of one String item by client index `ci` at visible pos p: `nb` UTF-8 bytes
 * of text that are `k` UTF-16 units long (the item's clock length, block.rs ItemContent::len) */
static void doc_insert_u(doc_t *d, bytes_t *out, uint32_t ci, uint64_t p, const uint8_t *text, uint32_t k,
                         uint32_t nb, const char *root) {
  int has_o = 0, has_r = 0;
  uint32_t oc = 0, ok = 0, rc = 0, rk = 0;
  size_t at = 0;
  if (p > 0) {
    uint64_t vis = 0;
    size_t i = 0;
    for (; i < d->n; i++) {
      if (d->r[i].del) continue;
      if (vis + d->r[i].len >= p) break;
      vis += d->r[i].len;
    }
    uint32_t o = (uint32_t)(p - vis);
    has_o = 1;
    oc = d->client_ids[d->r[i].cl];
    ok = d->r[i].clock + o - 1;
    if (o < d->r[i].len) runs_split(d, i, o);
    at = i + 1;
  }
  if (at < d->n) {
    has_r = 1;
    rc = d->client_ids[d->r[at].cl];
    rk = d->r[at].clock;
  }
  uint32_t clock = d->clocks[ci];
  run_t nr = {ci, clock, k, 0};
  runs_insert_at(d, at, nr);
  d->clocks[ci] += k;
  d->visible += k;
  /* v1 update */
  putv(out, 1);
  putv(out, 1);
  putv(out, d->client_ids[ci]);
  putv(out, clock);
  put(out, (uint8_t)((has_o ? 0x80 : 0) | (has_r ? 0x40 : 0) | 4));
  if (has_o) {
    putv(out, oc);
    putv(out, ok);
  }
  if (has_r) {
    putv(out, rc);
    putv(out, rk);
  }
  if (!has_o && !has_r) {
    putv(out, 1);
    size_t rl = strlen(root);
    putv(out, rl);
    putbytes(out, (const uint8_t *)root, rl);
  }
  putv(out, nb);
  putbytes(out, text, nb);
  putv(out, 0); /* empty DeleteSet */
}
static void doc_insert(doc_t *d, bytes_t *out, uint32_t ci, uint64_t p, const uint8_t *text, uint32_t k,
                       const char *root) {
  doc_insert_u(d, out, ci, p, text, k, k, root);
}

typedef struct {
  uint32_t client, clock, len;
} drange_t;
static int cmp_drange(const void *a, const void *b) {
  const drange_t *x = a, *y = b;
  if (x->client != y->client) return x->client > y->client ? -1 : 1; /* client desc */
  return x->clock < y->clock ? -1 : x->clock > y->clock;
}
/* delete k visible chars at p; emits a DS-only update */
static void doc_delete(doc_t *d, bytes_t *out, uint64_t p, uint64_t k, drange_t **scratch, size_t *scap) {
  uint64_t vis = 0;
  size_t nr = 0;
  for (size_t i = 0; i < d->n && k > 0; i++) {
    if (d->r[i].del) continue;
    uint32_t len = d->r[i].len;
    if (vis + len <= p) {
      vis += len;
      continue;
    }
    if (vis < p) { /* split off the head that stays */
      runs_split(d, i, (uint32_t)(p - vis));
      vis = p;
      continue; /* next iteration handles the tail run */
    }
    if (len > k) runs_split(d, i, (uint32_t)k);
    run_t *r = &d->r[i];
    r->del = 1;
    if (nr == *scap) {
      *scap = *scap ? *scap * 2 : 16;
      *scratch = realloc(*scratch, *scap * sizeof(drange_t));
    }
    (*scratch)[nr].client = d->client_ids[r->cl];
    (*scratch)[nr].clock = r->clock;
    (*scratch)[nr].len = r->len;
    nr++;
    k -= r->len;
    d->visible -= r->len;
    p += 0;
    vis += 0;
  }
  drange_t *rs = *scratch;
  qsort(rs, nr, sizeof(drange_t), cmp_drange);
  /* merge consecutive ranges of one client (Yjs sortAndMergeDeleteSet) */
  size_t m = 0;
  for (size_t i = 0; i < nr; i++) {
    if (m && rs[m - 1].client == rs[i].client && rs[m - 1].clock + rs[m - 1].len == rs[i].clock)
      rs[m - 1].len += rs[i].len;
    else
      rs[m++] = rs[i];
  }
  putv(out, 0); /* no blocks */
  size_t ncl = 0;
  for (size_t i = 0; i < m; i++)
    if (i == 0 || rs[i].client != rs[i - 1].client) ncl++;
  putv(out, ncl);
  for (size_t i = 0; i < m;) {
    size_t j = i;
    while (j < m && rs[j].client == rs[i].client) j++;
    putv(out, rs[i].client);
    putv(out, j - i);
    for (size_t q = i; q < j; q++) {
      putv(out, rs[q].clock);
      putv(out, rs[q].len);
    }
    i = j;
  }
}

static void doc_init(doc_t *d, uint64_t *rng, uint32_t n_clients) {
  memset(d, 0, sizeof(*d));
  d->n_clients = n_clients;
  d->client_ids = malloc(n_clients * sizeof(uint32_t));
  d->clocks = calloc(n_clients, sizeof(uint32_t));
  for (uint32_t c = 0; c < n_clients; c++) {
    uint32_t id;
    int dup;
    do {
      id = (uint32_t)splitmix64(rng) & 0x7FFFFFFF;
      dup = id == 0;
      for (uint32_t q = 0; q < c; q++) dup |= d->client_ids[q] == id;
    } while (dup);
    d->client_ids[c] = id;
  }
}
static void doc_free(doc_t *d) {
  free(d->r);
  free(d->client_ids);
  free(d->clocks);
}

/* ------------------------------------------------------------------ per-doc generation */
typedef struct {
  bytes_t bytes;
  uint64_t *ends; /* end offset (relative) of each update */
  size_t n_upd, cap_upd;
} docout_t;
static void mark_end(docout_t *o) {
  if (o->n_upd == o->cap_upd) {
    o->cap_upd = o->cap_upd ? o->cap_upd * 2 : 64;
    o->ends = realloc(o->ends, o->cap_upd * sizeof(uint64_t));
  }
  o->ends[o->n_upd++] = o->bytes.n;
}

typedef struct {
  int kind; /* 2 = text (C2/C3), 4 = delete-heavy with snapshot (C4) */
  uint64_t seed;
  const uint64_t *ids; /* global document ids (seed per doc), NULL = 0..n-1 */
  const uint32_t *n_ops;
  uint32_t min_clients, max_clients;
  double del_frac;
  docout_t *outs;
  size_t n_docs, next;
  pthread_mutex_t mu;
} gen_t;

static void gen_text_doc(gen_t *g, size_t di, docout_t *o) {
  uint64_t rng = g->seed ^ (g->ids ? g->ids[di] : (uint64_t)di);
  splitmix64(&rng);
  uint32_t nc = g->min_clients + urand(&rng, g->max_clients - g->min_clients + 1);
  doc_t d;
  doc_init(&d, &rng, nc);
  drange_t *scratch = NULL;
  size_t scap = 0;
  uint8_t text[16];
  for (uint32_t op = 0; op < g->n_ops[di]; op++) {
    uint32_t ci = urand(&rng, nc);
    double u = (double)(splitmix64(&rng) >> 11) / 9007199254740992.0;
    if (d.visible > 0 && u < g->del_frac) {
      uint64_t p = splitmix64(&rng) % d.visible;
      uint64_t k = 1 + urand(&rng, 5);
      if (k > d.visible - p) k = d.visible - p;
      doc_delete(&d, &o->bytes, p, k, &scratch, &scap);
    } else {
      uint32_t k = 1 + urand(&rng, 8);
      for (uint32_t q = 0; q < k; q++) text[q] = (uint8_t)('a' + urand(&rng, 26));
      uint64_t p = splitmix64(&rng) % (d.visible + 1);
      doc_insert(&d, &o->bytes, ci, p, text, k, "text");
    }
    mark_end(o);
  }
  free(scratch);
  doc_free(&d);
}

/* C4: snapshot (GC'd deleted runs + surviving item pieces) at half the log, then
 * the log with 10% of updates withheld and 5% stale duplicates */
typedef struct {
  uint32_t cl, clock, len, oc, ok, rc, rk;
  uint8_t has_o, has_r;
  uint8_t text[8];
} ins_t;
static void gen_c4_doc(gen_t *g, size_t di, docout_t *o) {
  uint64_t rng = g->seed ^ (g->ids ? g->ids[di] : (uint64_t)di);
  splitmix64(&rng);
  uint32_t nc = g->min_clients + urand(&rng, g->max_clients - g->min_clients + 1);
  doc_t d;
  doc_init(&d, &rng, nc);
  drange_t *scratch = NULL;
  size_t scap = 0;
  uint32_t nops = g->n_ops[di];
  bytes_t log = {0};
  uint64_t *ends = malloc((nops + 1) * sizeof(uint64_t));
  ins_t *ins = malloc((nops + 1) * sizeof(ins_t));
  size_t nins = 0;
  uint32_t snap_at = nops / 2;
  bytes_t snap = {0};
  for (uint32_t op = 0; op < nops; op++) {
    uint32_t ci = urand(&rng, nc);
    double u = (double)(splitmix64(&rng) >> 11) / 9007199254740992.0;
    if (d.visible > 0 && u < g->del_frac) {
      uint64_t p = splitmix64(&rng) % d.visible;
      uint64_t k = 1 + urand(&rng, 5);
      if (k > d.visible - p) k = d.visible - p;
      doc_delete(&d, &log, p, k, &scratch, &scap);
    } else {
      uint32_t k = 1 + urand(&rng, 8);
      uint8_t text[8];
      for (uint32_t q = 0; q < k; q++) text[q] = (uint8_t)('a' + urand(&rng, 26));
      uint64_t p = splitmix64(&rng) % (d.visible + 1);
      size_t before = log.n;
      doc_insert(&d, &log, ci, p, text, k, "text");
      /* remember the item (parse our own emitted header back) */
      ins_t it;
      memset(&it, 0, sizeof(it));
      it.cl = ci;
      it.clock = d.clocks[ci] - k;
      it.len = k;
      memcpy(it.text, text, k);
      const uint8_t *b = log.d + before;
      size_t i = 0;
#define GETV(v)                                                                                    \
  do {                                                                                             \
    uint64_t _v = 0;                                                                               \
    int _s = 0;                                                                                    \
    for (;;) {                                                                                     \
      uint8_t _x = b[i++];                                                                         \
      _v |= (uint64_t)(_x & 0x7f) << _s;                                                           \
      _s += 7;                                                                                     \
      if (_x < 0x80) break;                                                                        \
    }                                                                                              \
    v = (uint32_t)_v;                                                                              \
  } while (0)
      uint32_t v;
      GETV(v);
      GETV(v);
      GETV(v);
      GETV(v);
      uint8_t info = b[i++];
      if (info & 0x80) {
        it.has_o = 1;
        GETV(it.oc);
        GETV(it.ok);
      }
      if (info & 0x40) {
        it.has_r = 1;
        GETV(it.rc);
        GETV(it.rk);
      }
#undef GETV
      ins[nins++] = it;
    }
    ends[op] = log.n;
    if (op + 1 == snap_at) {
      /* snapshot: per client (desc id), clock order; deleted chars -> merged GC */
      uint32_t *order = malloc(nc * sizeof(uint32_t));
      for (uint32_t c = 0; c < nc; c++) order[c] = c;
      for (uint32_t a = 1; a < nc; a++)
        for (uint32_t b2 = a; b2 > 0 && d.client_ids[order[b2]] > d.client_ids[order[b2 - 1]]; b2--) {
          uint32_t t = order[b2];
          order[b2] = order[b2 - 1];
          order[b2 - 1] = t;
        }
      /* deleted flag per (client, clock) from the run list */
      uint8_t **deleted = malloc(nc * sizeof(uint8_t *));
      for (uint32_t c = 0; c < nc; c++) deleted[c] = calloc(d.clocks[c] + 1, 1);
      for (size_t i = 0; i < d.n; i++)
        if (d.r[i].del)
          for (uint32_t q = 0; q < d.r[i].len; q++) deleted[d.r[i].cl][d.r[i].clock + q] = 1;
      uint32_t ncl_nonempty = 0;
      for (uint32_t c = 0; c < nc; c++) ncl_nonempty += d.clocks[c] > 0;
      putv(&snap, ncl_nonempty);
      for (uint32_t oi = 0; oi < nc; oi++) {
        uint32_t c = order[oi];
        if (!d.clocks[c]) continue;
        bytes_t body = {0};
        uint32_t nblocks = 0;
        uint32_t gc_start = 0, gc_len = 0;
        for (size_t k2 = 0; k2 < nins; k2++) {
          ins_t *it = &ins[k2];
          if (it->cl != c) continue;
          for (uint32_t q = 0; q < it->len;) {
            if (deleted[c][it->clock + q]) {
              if (!gc_len) gc_start = it->clock + q;
              gc_len++;
              q++;
              continue;
            }
            if (gc_len) {
              put(&body, 0);
              putv(&body, gc_len);
              nblocks++;
              gc_len = 0;
            }
            uint32_t q2 = q;
            while (q2 < it->len && !deleted[c][it->clock + q2]) q2++;
            /* item piece [q, q2) */
            int has_o = q > 0 ? 1 : it->has_o;
            int has_r = q2 == it->len ? it->has_r : 0;
            if (q2 < it->len) has_r = it->has_r; /* right origin kept (slice.rs:215) */
            put(&body, (uint8_t)((has_o ? 0x80 : 0) | (has_r ? 0x40 : 0) | 4));
            if (has_o) {
              putv(&body, q > 0 ? d.client_ids[c] : it->oc);
              putv(&body, q > 0 ? it->clock + q - 1 : it->ok);
            }
            if (has_r) {
              putv(&body, it->rc);
              putv(&body, it->rk);
            }
            if (!has_o && !has_r) {
              putv(&body, 1);
              putv(&body, 4);
              putbytes(&body, (const uint8_t *)"text", 4);
            }
            putv(&body, q2 - q);
            putbytes(&body, it->text + q, q2 - q);
            nblocks++;
            q = q2;
          }
        }
        if (gc_len) {
          put(&body, 0);
          putv(&body, gc_len);
          nblocks++;
        }
        (void)gc_start;
        putv(&snap, nblocks);
        putv(&snap, d.client_ids[c]);
        putv(&snap, 0);
        putbytes(&snap, body.d, body.n);
        free(body.d);
      }
      /* snapshot DeleteSet: every deleted range, client desc */
      uint32_t nds = 0;
      for (uint32_t oi = 0; oi < nc; oi++) {
        uint32_t c = order[oi];
        for (uint32_t q = 0; q < d.clocks[c]; q++)
          if (deleted[c][q] && (q == 0 || !deleted[c][q - 1])) {
            nds++;
            break;
          }
      }
      putv(&snap, nds);
      for (uint32_t oi = 0; oi < nc; oi++) {
        uint32_t c = order[oi];
        uint32_t nr = 0;
        for (uint32_t q = 0; q < d.clocks[c]; q++) nr += deleted[c][q] && (q == 0 || !deleted[c][q - 1]);
        if (!nr) continue;
        putv(&snap, d.client_ids[c]);
        putv(&snap, nr);
        for (uint32_t q = 0; q < d.clocks[c];) {
          if (!deleted[c][q]) {
            q++;
            continue;
          }
          uint32_t q2 = q;
          while (q2 < d.clocks[c] && deleted[c][q2]) q2++;
          putv(&snap, q);
          putv(&snap, q2 - q);
          q = q2;
        }
      }
      for (uint32_t c = 0; c < nc; c++) free(deleted[c]);
      free(deleted);
      free(order);
    }
  }
  /* assemble: snapshot, then the log with 10% withheld and 5% duplicated */
  putbytes(&o->bytes, snap.d, snap.n);
  mark_end(o);
  for (uint32_t op = 0; op < nops; op++) {
    uint64_t s = op ? ends[op - 1] : 0, e = ends[op];
    uint32_t r = urand(&rng, 100);
    if (r < 10) continue;
    putbytes(&o->bytes, log.d + s, e - s);
    mark_end(o);
    if (r >= 95) {
      putbytes(&o->bytes, log.d + s, e - s);
      mark_end(o);
    }
  }
  free(snap.d);
  free(log.d);
  free(ends);
  free(ins);
  free(scratch);
  doc_free(&d);
}

static void *gen_worker(void *arg) {
  gen_t *g = arg;
  for (;;) {
    pthread_mutex_lock(&g->mu);
    size_t d0 = g->next;
    g->next += 16;
    pthread_mutex_unlock(&g->mu);
    if (d0 >= g->n_docs) break;
    for (size_t di = d0; di < d0 + 16 && di < g->n_docs; di++) {
      if (g->kind == 4)
        gen_c4_doc(g, di, &g->outs[di]);
      else
        gen_text_doc(g, di, &g->outs[di]);
    }
  }
  return NULL;
}

/* Generates n_docs documents; outputs malloc'd arena, upd_off[n_upd+1], doc_upd[n_docs+1]. */
int yw_generate_ids(int kind, uint64_t seed, size_t n_docs, const uint64_t *ids, const uint32_t *n_ops,
                    uint32_t min_clients, uint32_t max_clients, double del_frac, int threads, uint8_t **bytes,
                    uint64_t *n_bytes, uint64_t **upd_off, uint64_t *n_upd, uint64_t **doc_upd);
int yw_generate(int kind, uint64_t seed, size_t n_docs, const uint32_t *n_ops, uint32_t min_clients,
                uint32_t max_clients, double del_frac, int threads, uint8_t **bytes, uint64_t *n_bytes,
                uint64_t **upd_off, uint64_t *n_upd, uint64_t **doc_upd) {
  return yw_generate_ids(kind, seed, n_docs, NULL, n_ops, min_clients, max_clients, del_frac, threads, bytes,
                         n_bytes, upd_off, n_upd, doc_upd);
}
/* splitmix64 finaliser used for doc-hash sharding (shard = yw_doc_hash(id) % G) */
uint64_t yw_doc_hash(uint64_t id) {
  uint64_t s = id;
  return splitmix64(&s);
}
int yw_generate_ids(int kind, uint64_t seed, size_t n_docs, const uint64_t *ids, const uint32_t *n_ops,
                    uint32_t min_clients, uint32_t max_clients, double del_frac, int threads, uint8_t **bytes,
                    uint64_t *n_bytes, uint64_t **upd_off, uint64_t *n_upd, uint64_t **doc_upd) {
  gen_t g;
  memset(&g, 0, sizeof(g));
  g.ids = ids;
  g.kind = kind;
  g.seed = seed;
  g.n_ops = n_ops;
  g.min_clients = min_clients;
  g.max_clients = max_clients;
  g.del_frac = del_frac;
  g.n_docs = n_docs;
  g.outs = calloc(n_docs + 1, sizeof(docout_t));
  pthread_mutex_init(&g.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t *th = malloc(threads * sizeof(pthread_t));
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, gen_worker, &g);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&g.mu);
  uint64_t tb = 0, tu = 0;
  for (size_t di = 0; di < n_docs; di++) {
    tb += g.outs[di].bytes.n;
    tu += g.outs[di].n_upd;
  }
  *bytes = malloc(tb + 1);
  *upd_off = malloc((tu + 1) * sizeof(uint64_t));
  *doc_upd = malloc((n_docs + 1) * sizeof(uint64_t));
  uint64_t pb = 0, pu = 0;
  for (size_t di = 0; di < n_docs; di++) {
    docout_t *o = &g.outs[di];
    (*doc_upd)[di] = pu;
    if (o->bytes.n) memcpy(*bytes + pb, o->bytes.d, o->bytes.n);
    uint64_t prev = 0;
    for (size_t u = 0; u < o->n_upd; u++) {
      (*upd_off)[pu++] = pb + prev;
      prev = o->ends[u];
    }
    pb += o->bytes.n;
    free(o->bytes.d);
    free(o->ends);
  }
  (*upd_off)[pu] = pb;
  (*doc_upd)[n_docs] = pu;
  *n_bytes = tb;
  *n_upd = tu;
  free(g.outs);
  return 0;
}

/* C1: replay an editing trace (ops = pos, del, ins_len bytes, ins_units UTF-16 units (NULL:
 * ASCII, = ins_len), then ins bytes) as one doc, client id `client`, one update per patch
 * (a patch that deletes and inserts gives one update: its block, then its DeleteSet).
 * Positions and delete counts are UTF-16 units. */
int yw_replay(const uint32_t *pos, const uint32_t *del, const uint32_t *ins_len, const uint32_t *ins_units,
              const uint8_t *ins_bytes, size_t n_txn, uint32_t client, uint8_t **bytes, uint64_t *n_bytes,
              uint64_t **upd_off) {
  doc_t d;
  memset(&d, 0, sizeof(d));
  d.n_clients = 1;
  d.client_ids = malloc(sizeof(uint32_t));
  d.clocks = calloc(1, sizeof(uint32_t));
  d.client_ids[0] = client;
  bytes_t out = {0}, tmp = {0};
  uint64_t *offs = malloc((n_txn + 1) * sizeof(uint64_t));
  drange_t *scratch = NULL;
  size_t scap = 0, ib = 0;
  for (size_t t = 0; t < n_txn; t++) {
    offs[t] = out.n;
    if (del[t] && ins_len[t]) {
      /* delete first (it fixes positions), then insert; emit one update [block][DS] */
      tmp.n = 0;
      doc_delete(&d, &tmp, pos[t], del[t], &scratch, &scap);
      bytes_t blk = {0};
      doc_insert_u(&d, &blk, 0, pos[t], ins_bytes + ib, ins_units ? ins_units[t] : ins_len[t], ins_len[t], "text");
      putbytes(&out, blk.d, blk.n - 1); /* drop the empty DS byte */
      putbytes(&out, tmp.d + 1, tmp.n - 1); /* drop the "0 clients" byte */
      free(blk.d);
    } else if (del[t]) {
      doc_delete(&d, &out, pos[t], del[t], &scratch, &scap);
    } else {
      doc_insert_u(&d, &out, 0, pos[t], ins_bytes + ib, ins_units ? ins_units[t] : ins_len[t], ins_len[t], "text");
    }
    ib += ins_len[t];
  }
  offs[n_txn] = out.n;
  *bytes = out.d;
  *n_bytes = out.n;
  *upd_off = offs;
  free(tmp.d);
  free(scratch);
  doc_free(&d);
  return 0;
}

void yw_free(void *p) { free(p); }
