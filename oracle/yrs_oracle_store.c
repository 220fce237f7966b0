/*
 * yrs_oracle_store.c — TEST INFRASTRUCTURE ONLY (included by yrs_oracle.c): a CPU restatement
 * of store-based compaction in yrs — a Doc with default options (GC on) applies a document's
 * v1 updates in order, one transaction each (TransactionMut::apply_update + commit,
 * yrs/src/transaction.rs:664-726, 828-910), then encode_state_as_update_v1 with an empty
 * state vector (transaction.rs:73-85, store.rs:194-232, merge_pending_v1 transaction.rs:247-263).
 *
 * Restated here:
 *   Update::integrate          yrs/src/update.rs:169-308 (stack of missing dependencies,
 *                              pending blocks, missing(): :310-345, return_stack: :411-431)
 *   Item::repair / integrate   yrs/src/block.rs:1287-1350, 482-771 (YATA conflict loop,
 *                              parent / parent_sub, map values, parent lengths)
 *   ItemPtr::splice            block.rs:435-478; ItemContent::splice / try_squash 1837-1906
 *   BlockStore                 yrs/src/block_store.rs (find_pivot :70-96, split_block :456-475,
 *                              get_item_clean_start / end :402-416, squash_left :243-271,
 *                              squash_left_range_compaction :155-241)
 *   TransactionMut::apply_delete / delete      transaction.rs:472-578, 579-662
 *   GC                         yrs/src/gc.rs:10-66, block.rs:1371-1382, 1907-1926
 *   DeleteSet::try_squash_with yrs/src/id_set.rs:571-598; DeleteSet from the store :448-468
 * Content kinds: Deleted, JSON, Binary, String, Embed, Format, Any and nested types
 * (TypeRef other than WeakLink); Move, Doc and WeakLink contents return UNSUPPORTED.
 * Offsets are UTF-16 (yrs integrates remote updates with OffsetKind::Utf16).
 */

/* ------------------------------------------------------------------ model */
typedef VEC(uint32_t) u32vec_t;
typedef struct {
  uint64_t client;
  uint32_t clock, len;
  int32_t left, right;  /* neighbours in the parent's sequence (item index, -1 none) */
  uint8_t has_origin, has_ro;
  uint64_t oc, rc;
  uint32_t ok, rk;
  int32_t parent;       /* branch index; -1 = TypePtr::Unknown */
  uint8_t pkind;        /* decoded parent before repair: PK_NAMED / PK_ID / PK_UNKNOWN */
  uint64_t pc;
  uint32_t pk;
  span_t pname;
  uint8_t has_psub;
  span_t psub;
  uint8_t deleted, countable, keep;
  uint8_t ref;          /* content ref: 1 Deleted, 2 JSON, 3 Binary, 4 String, 5 Embed, 6 Format, 7 Type, 8 Any */
  VEC(uint8_t) str;     /* String bytes (owned) */
  VEC(span_t) el;       /* Any / JSON element spans (input buffers stay alive) */
  span_t cs, cs2;       /* Binary, Embed JSON, Format key + JSON, XmlElement name */
  uint8_t tref;
  int32_t branch;       /* Type: its branch */
  uint32_t mk_ibo, mk_conf; /* YATA loop set membership (generation stamps) */
} sitem_t;

typedef struct {
  uint8_t gc;
  int32_t item;
  uint32_t start, end; /* GC: clocks [start, end] */
} cell_t;
typedef struct {
  VEC(cell_t) v;
} slist_t;

typedef struct {
  int32_t start, item; /* first item of the sequence; owning item (nested) or -1 (root) */
  span_t name;
  VEC(span_t) keys;    /* map: parent_sub -> current value (rightmost item) */
  VEC(int32_t) vals;
} branch_t;

typedef struct {
  uint64_t client;
  uint32_t clock;
} sid_t;
typedef VEC(sid_t) sidvec_t;

typedef struct {
  VEC(sitem_t) it;
  hb_t clients; /* BlockStore.clients: HashMap<ClientID, ClientBlockList> (iteration order) */
  VEC(slist_t) lists;
  VEC(branch_t) br;
  /* pending update (encoded v1) + its missing state vector; pending delete set (encoded [0] + DS) */
  VEC(uint8_t) pend;
  int has_pend;
  hb_t pmiss;
  u32vec_t pmiss_clock;
  VEC(uint8_t) pend_ds;
  int has_pend_ds;
  /* buffers items may point into (decoded updates, merged pending updates) */
  VEC(uint8_t *) owned;
  /* the current transaction */
  hb_t before;
  u32vec_t before_clock;
  hb_t tds; /* txn.delete_set */
  idrvec_t tdsv;
  sidvec_t merge_blocks;
  uint32_t gen_ibo, gen_conf;
  int err;
} sdoc_t;

static slist_t *s_list(sdoc_t *d, uint64_t client) {
  int32_t e = hb_find(&d->clients, client);
  return e >= 0 ? &d->lists.d[e] : NULL;
}
/* get_client_blocks_mut: entry().or_insert */
static slist_t *s_list_mut(sdoc_t *d, uint64_t client) {
  bool ex;
  int32_t e = hb_entry(&d->clients, client, &ex);
  if (!ex) {
    slist_t l = {0};
    VPUSH(d->lists, l);
  }
  return &d->lists.d[e];
}
static uint32_t cell_start(const sdoc_t *d, const cell_t *c) { return c->gc ? c->start : d->it.d[c->item].clock; }
static uint32_t cell_end(const sdoc_t *d, const cell_t *c) {
  return c->gc ? c->end : d->it.d[c->item].clock + d->it.d[c->item].len - 1;
}
static bool cell_deleted(const sdoc_t *d, const cell_t *c) { return c->gc || d->it.d[c->item].deleted; }
/* ClientBlockList::clock: end of the last block */
static uint32_t s_clock(const sdoc_t *d, uint64_t client) {
  slist_t *l = s_list((sdoc_t *)d, client);
  if (!l || !l->v.n) return 0;
  return cell_end(d, &l->v.d[l->v.n - 1]) + 1;
}
/* find_pivot (block_store.rs:70-96): index of the block containing clock, or -1 */
static int64_t s_pivot(const sdoc_t *d, const slist_t *l, uint32_t clock) {
  if (!l || !l->v.n) return -1;
  int64_t lo = 0, hi = (int64_t)l->v.n - 1;
  while (lo <= hi) {
    int64_t mid = (lo + hi) / 2;
    uint32_t s = cell_start(d, &l->v.d[mid]), e = cell_end(d, &l->v.d[mid]);
    if (s <= clock) {
      if (clock <= e) return mid;
      lo = mid + 1;
    } else
      hi = mid - 1;
  }
  return -1;
}
/* BlockStore::get_item: the Item (not GC) containing id */
static int32_t s_get_item(sdoc_t *d, uint64_t client, uint32_t clock) {
  slist_t *l = s_list(d, client);
  int64_t i = s_pivot(d, l, clock);
  if (i < 0 || l->v.d[i].gc) return -1;
  return l->v.d[i].item;
}
static void s_list_insert(slist_t *l, size_t at, cell_t c) {
  VPUSH(l->v, c);
  memmove(l->v.d + at + 1, l->v.d + at, (l->v.n - 1 - at) * sizeof(cell_t));
  l->v.d[at] = c;
}

/* ------------------------------------------------------------------ content */
static uint32_t sc_len(const sitem_t *x) {
  switch (x->ref) {
  case 1: return x->len; /* Deleted(n): len kept in x->len */
  case 4: return x->str.n == 1 ? 1 : str_len16(x->str.d, (uint32_t)x->str.n);
  case 2: case 8: return (uint32_t)x->el.n;
  default: return 1;
  }
}
/* ItemContent::splice(offset, Utf16) (block.rs:1837-1879): x keeps [0, off), *r gets the rest.
 * Contents of length 1 cannot be split: yrs unwraps None -> panic. */
static int sc_split(sitem_t *x, uint32_t off, sitem_t *r) {
  switch (x->ref) {
  case 1: r->len = x->len - off; return 0;
  case 4: {
    uint32_t bo;
    TRY(str_split16(x->str.d, (uint32_t)x->str.n, off, &bo));
    for (size_t i = bo; i < x->str.n; i++) VPUSH(r->str, x->str.d[i]);
    x->str.n = bo;
    return 0;
  }
  case 2: case 8:
    for (size_t i = off; i < x->el.n; i++) VPUSH(r->el, x->el.d[i]);
    x->el.n = off;
    return 0;
  default: return YO_ERR_REFERENCE_PANIC;
  }
}
/* ItemContent::try_squash (block.rs:1884-1906) */
static bool sc_try_squash(sitem_t *a, const sitem_t *b) {
  if (a->ref != b->ref) return false;
  switch (a->ref) {
  case 8: case 2:
    for (size_t i = 0; i < b->el.n; i++) VPUSH(a->el, b->el.d[i]);
    return true;
  case 1: a->len += b->len; return true; /* Deleted counts (len is recomputed by the caller) */
  case 4:
    for (size_t i = 0; i < b->str.n; i++) VPUSH(a->str, b->str.d[i]);
    return true;
  default: return false;
  }
}
static bool sc_countable(uint8_t ref) { return ref != 1 && ref != 6; } /* Deleted / Format are not */

/* ------------------------------------------------------------------ splits (block.rs:435-478) */
static int32_t s_new_item(sdoc_t *d) {
  sitem_t z;
  memset(&z, 0, sizeof(z));
  z.left = z.right = z.parent = z.branch = -1;
  VPUSH(d->it, z);
  return (int32_t)d->it.n - 1;
}
static void br_map_set(sdoc_t *d, int32_t b, span_t key, int32_t v) {
  branch_t *B = &d->br.d[b];
  for (size_t i = 0; i < B->keys.n; i++)
    if (B->keys.d[i].n == key.n && !memcmp(B->keys.d[i].p, key.p, key.n)) {
      B->vals.d[i] = v;
      return;
    }
  VPUSH(B->keys, key);
  VPUSH(B->vals, v);
}
static int32_t br_map_get(sdoc_t *d, int32_t b, span_t key) {
  branch_t *B = &d->br.d[b];
  for (size_t i = 0; i < B->keys.n; i++)
    if (B->keys.d[i].n == key.n && !memcmp(B->keys.d[i].p, key.p, key.n)) return B->vals.d[i];
  return -1;
}
/* ItemPtr::splice + BlockStore::split_block (insert at pivot + 1): returns the right part */
static int32_t s_split(sdoc_t *d, int32_t xi, uint32_t off) {
  if (off == 0) return -1;
  int32_t ri = s_new_item(d);
  sitem_t *x = &d->it.d[xi], *r = &d->it.d[ri];
  r->ref = x->ref;
  int e = sc_split(x, off, r);
  if (e) {
    d->err = e;
    return -1;
  }
  r->client = x->client;
  r->clock = x->clock + off;
  if (x->ref == 1) x->len = off;
  r->len = sc_len(r);
  r->left = xi;
  r->right = x->right;
  r->has_origin = 1;
  r->oc = x->client;
  r->ok = x->clock + off - 1;
  r->has_ro = x->has_ro;
  r->rc = x->rc;
  r->rk = x->rk;
  r->parent = x->parent;
  r->pkind = x->pkind;
  r->pc = x->pc;
  r->pk = x->pk;
  r->pname = x->pname;
  r->has_psub = x->has_psub;
  r->psub = x->psub;
  r->deleted = x->deleted;
  r->countable = x->countable;
  r->keep = x->keep;
  r->cs = x->cs;
  r->cs2 = x->cs2;
  r->tref = x->tref;
  x->len = off;
  if (x->right >= 0) d->it.d[x->right].left = ri;
  if (x->has_psub && x->right < 0 && x->parent >= 0) br_map_set(d, x->parent, x->psub, ri);
  x->right = ri;
  slist_t *l = s_list(d, x->client);
  int64_t p = s_pivot(d, l, x->clock);
  cell_t c = {0, ri, 0, 0};
  s_list_insert(l, (size_t)p + 1, c);
  return ri;
}
/* get_item_clean_start + materialize: the item starting exactly at id */
static int32_t s_clean_start(sdoc_t *d, uint64_t client, uint32_t clock) {
  int32_t xi = s_get_item(d, client, clock);
  if (xi < 0) return -1;
  uint32_t off = clock - d->it.d[xi].clock;
  if (off == 0) return xi;
  return s_split(d, xi, off);
}
/* get_item_clean_end + materialize: the item ending exactly at id */
static int32_t s_clean_end(sdoc_t *d, uint64_t client, uint32_t clock) {
  int32_t xi = s_get_item(d, client, clock);
  if (xi < 0) return -1;
  uint32_t off = clock - d->it.d[xi].clock;
  if (off + 1 < d->it.d[xi].len) s_split(d, xi, off + 1);
  return xi;
}

/* ------------------------------------------------------------------ types */
static int32_t s_root(sdoc_t *d, span_t name) { /* Store::get_or_create_type */
  for (size_t i = 0; i < d->br.n; i++)
    if (d->br.d[i].item < 0 && d->br.d[i].name.n == name.n && !memcmp(d->br.d[i].name.p, name.p, name.n))
      return (int32_t)i;
  branch_t b;
  memset(&b, 0, sizeof(b));
  b.start = -1;
  b.item = -1;
  b.name = name;
  VPUSH(d->br, b);
  return (int32_t)d->br.n - 1;
}

/* ------------------------------------------------------------------ transaction */
/* IdRange::push (id_set.rs:95-123) */
static void idr_push(idr_t *g, rng_t r) {
  if (g->cont) {
    if (g->c.e >= r.s) {
      if (g->c.s > r.e) {
        rng_t a = g->c;
        g->cont = 0;
        g->v.n = 0;
        VPUSH(g->v, r);
        VPUSH(g->v, a);
      } else {
        if (r.e > g->c.e) g->c.e = r.e;
        if (r.s < g->c.s) g->c.s = r.s;
      }
    } else {
      rng_t a = g->c;
      g->cont = 0;
      g->v.n = 0;
      VPUSH(g->v, a);
      VPUSH(g->v, r);
    }
  } else if (g->v.n == 0) {
    g->cont = 1;
    g->c = r;
  } else {
    rng_t *last = &g->v.d[g->v.n - 1];
    if (rng_disjoint(*last, r))
      VPUSH(g->v, r);
    else {
      if (r.s < last->s) last->s = r.s;
      if (r.e > last->e) last->e = r.e;
    }
  }
}
/* IdSet::insert (id_set.rs:368-378): a vacant client gets Continuous(range) */
static void idset_insert(hb_t *t, idrvec_t *v, uint64_t client, uint32_t clock, uint32_t len) {
  bool ex;
  int32_t e = hb_entry(t, client, &ex);
  rng_t r = {clock, clock + len};
  if (!ex) {
    idr_t g;
    memset(&g, 0, sizeof(g));
    g.cont = 1;
    g.c = r;
    VPUSH(*v, g);
    return;
  }
  idr_push(&v->d[e], r);
}
static void t_ds_insert(sdoc_t *d, uint64_t client, uint32_t clock, uint32_t len) {
  idset_insert(&d->tds, (idrvec_t *)&d->tdsv, client, clock, len);
}
static bool s_parent_deleted(sdoc_t *d, int32_t b) {
  return b >= 0 && d->br.d[b].item >= 0 && d->it.d[d->br.d[b].item].deleted;
}
/* TransactionMut::delete (transaction.rs:579-662) */
static bool t_delete(sdoc_t *d, int32_t xi) {
  sitem_t *x = &d->it.d[xi];
  bool result = false;
  VEC(int32_t) rec = {0};
  if (!x->deleted) {
    x->deleted = 1;
    t_ds_insert(d, x->client, x->clock, x->len);
    if (x->ref == 7 && x->branch >= 0) {
      branch_t *B = &d->br.d[x->branch];
      for (int32_t p = B->start; p >= 0; p = d->it.d[p].right)
        if (!d->it.d[p].deleted) VPUSH(rec, p);
      for (size_t i = 0; i < B->vals.n; i++) VPUSH(rec, B->vals.d[i]);
    }
    result = true;
  }
  for (size_t i = 0; i < rec.n; i++) {
    sid_t id = {d->it.d[rec.d[i]].client, d->it.d[rec.d[i]].clock};
    if (!t_delete(d, rec.d[i])) VPUSH(d->merge_blocks, id);
  }
  VFREE(rec);
  return result;
}

/* ------------------------------------------------------------------ integrate (block.rs:482-771) */
static int32_t s_origin_item(sdoc_t *d, const sitem_t *x) {
  return x->has_origin ? s_get_item(d, x->oc, x->ok) : -1;
}
static bool s_same_origin(const sitem_t *a, const sitem_t *b) {
  return a->has_origin == b->has_origin && (!a->has_origin || (a->oc == b->oc && a->ok == b->ok));
}
static bool s_same_ro(const sitem_t *a, const sitem_t *b) {
  return a->has_ro == b->has_ro && (!a->has_ro || (a->rc == b->rc && a->rk == b->rk));
}
/* returns 1 = the block must be deleted after being added (should_delete) */
static int s_integrate(sdoc_t *d, int32_t xi, uint32_t offset) {
  sitem_t *x = &d->it.d[xi];
  if (offset > 0) {
    x->clock += offset;
    x->left = s_clean_end(d, x->client, x->clock - 1);
    x = &d->it.d[xi];
    if (x->left >= 0) {
      const sitem_t *l = &d->it.d[x->left];
      x->has_origin = 1;
      x->oc = l->client;
      x->ok = l->clock + l->len - 1;
    } else
      x->has_origin = 0;
    /* content.splice(offset, Utf16).unwrap(): the item keeps the right part */
    sitem_t tmp;
    memset(&tmp, 0, sizeof(tmp));
    tmp.ref = x->ref;
    int e = sc_split(x, offset, &tmp);
    if (e) {
      d->err = e;
      return 0;
    }
    VFREE(x->str);
    VFREE(x->el);
    x->str = tmp.str;
    x->el = tmp.el;
    if (x->ref == 1) x->len = x->len - offset;
    else x->len -= offset;
  }
  x = &d->it.d[xi];
  int32_t parent = x->parent;
  if (parent < 0) return 1; /* TypePtr::Unknown */
  int32_t left = x->left, right = x->right;
  bool right_null_or_has_left = right < 0 || d->it.d[right].left >= 0;
  bool left_other_right = left >= 0 && d->it.d[left].right != right;
  if ((left < 0 && right_null_or_has_left) || left_other_right) {
    int32_t o;
    if (left >= 0)
      o = d->it.d[left].right;
    else if (x->has_psub) {
      o = br_map_get(d, parent, x->psub);
      while (o >= 0 && d->it.d[o].left >= 0) o = d->it.d[o].left;
    } else
      o = d->br.d[parent].start;
    int32_t nl = x->left;
    uint32_t gi = ++d->gen_ibo;
    uint32_t gc = ++d->gen_conf;
    while (o >= 0 && o != x->right) {
      sitem_t *it = &d->it.d[o];
      it->mk_ibo = gi;
      it->mk_conf = gc;
      if (s_same_origin(x, it)) {
        if (it->client < x->client) {
          nl = o;
          gc = ++d->gen_conf; /* conflicting_items.clear() */
        } else if (s_same_ro(x, it)) {
          break;
        }
      } else {
        int32_t op = s_origin_item(d, it);
        if (op >= 0) {
          if (d->it.d[op].mk_ibo == gi) {
            if (d->it.d[op].mk_conf != gc) {
              nl = o;
              gc = ++d->gen_conf;
            }
          } else
            break;
        } else
          break;
      }
      o = d->it.d[o].right;
      x = &d->it.d[xi];
    }
    x = &d->it.d[xi];
    x->left = nl;
  }
  x = &d->it.d[xi];
  if (!x->has_psub) { /* inherit parent_sub from the neighbours */
    if (x->left >= 0) {
      if (d->it.d[x->left].has_psub) {
        x->has_psub = 1;
        x->psub = d->it.d[x->left].psub;
      } else if (x->right >= 0) {
        x->has_psub = d->it.d[x->right].has_psub;
        x->psub = d->it.d[x->right].psub;
      }
    }
  }
  /* reconnect left / right */
  if (x->left >= 0) {
    sitem_t *l = &d->it.d[x->left];
    x->right = l->right;
    l->right = xi;
  } else {
    int32_t r;
    if (x->has_psub) {
      r = br_map_get(d, parent, x->psub);
      while (r >= 0 && d->it.d[r].left >= 0) r = d->it.d[r].left;
    } else {
      r = d->br.d[parent].start;
      d->br.d[parent].start = xi;
    }
    x->right = r;
  }
  if (x->right >= 0) {
    d->it.d[x->right].left = xi;
  } else if (x->has_psub) {
    br_map_set(d, parent, x->psub, xi);
    if (x->left >= 0) t_delete(d, x->left); /* the previous value of the key */
  }
  x = &d->it.d[xi];
  if (x->ref == 1) { /* ItemContent::Deleted */
    t_ds_insert(d, x->client, x->clock, x->len);
    x->deleted = 1;
  }
  if (x->ref == 7) { /* ItemContent::Type: the nested branch */
    branch_t b;
    memset(&b, 0, sizeof(b));
    b.start = -1;
    b.item = xi;
    VPUSH(d->br, b);
    d->it.d[xi].branch = (int32_t)d->br.n - 1;
  }
  x = &d->it.d[xi];
  if (s_parent_deleted(d, parent) || (x->has_psub && x->right >= 0)) return 1;
  return 0;
}

/* Item::repair (block.rs:1287-1350) */
static void s_repair(sdoc_t *d, int32_t xi) {
  sitem_t *x = &d->it.d[xi];
  if (x->has_origin) {
    int32_t l = s_clean_end(d, x->oc, x->ok);
    d->it.d[xi].left = l;
  }
  x = &d->it.d[xi];
  if (x->has_ro) {
    int32_t r = s_clean_start(d, x->rc, x->rk);
    d->it.d[xi].right = r;
  }
  x = &d->it.d[xi];
  if (x->pkind == PK_NAMED) {
    x->parent = s_root(d, x->pname);
  } else if (x->pkind == PK_ID) {
    int32_t p = s_get_item(d, x->pc, x->pk);
    x = &d->it.d[xi];
    if (p >= 0 && d->it.d[p].ref == 7)
      x->parent = d->it.d[p].branch;
    else if (p >= 0 && d->it.d[p].ref == 1)
      x->parent = -1;
    else if (p >= 0)
      d->err = YO_ERR_REFERENCE_PANIC; /* "parent points to a block which is not a shared type" */
    else
      x->parent = -1;
  } else { /* TypePtr::Unknown: from the neighbours */
    x->parent = -1;
    if (x->left >= 0 && d->it.d[x->left].parent >= 0) {
      x->parent = d->it.d[x->left].parent;
      x->has_psub = d->it.d[x->left].has_psub;
      x->psub = d->it.d[x->left].psub;
    } else if (x->right >= 0 && d->it.d[x->right].parent >= 0) {
      x->parent = d->it.d[x->right].parent;
      x->has_psub = d->it.d[x->right].has_psub;
      x->psub = d->it.d[x->right].psub;
    }
  }
}

/* an Item from a decoded block */
static int s_item_from(sdoc_t *d, const upd_t *u, const blk_t *b, int32_t *out) {
  if (b->ref == 9 || b->ref == 11 || (b->ref == 7 && b->tref == 7) || b->ref > 11) return YO_ERR_UNSUPPORTED;
  int32_t xi = s_new_item(d);
  sitem_t *x = &d->it.d[xi];
  x->client = b->client;
  x->clock = b->clock;
  x->len = b->len;
  x->has_origin = b->has_origin;
  x->oc = b->oc;
  x->ok = b->ok;
  x->has_ro = b->has_ro;
  x->rc = b->rc;
  x->rk = b->rk;
  x->pkind = b->pkind;
  x->pc = b->pc;
  x->pk = b->pk;
  x->pname = b->pname;
  x->has_psub = b->has_psub;
  x->psub = b->psub;
  x->ref = b->ref;
  x->countable = sc_countable(b->ref);
  x->cs = b->cs;
  x->cs2 = b->cs2;
  x->tref = b->tref;
  if (b->ref == 4)
    for (uint32_t i = 0; i < b->cs.n; i++) VPUSH(x->str, b->cs.p[i]);
  if (b->ref == 2 || b->ref == 8)
    for (uint32_t i = 0; i < b->n; i++) VPUSH(x->el, u->elems.d[b->e0 + i]);
  *out = xi;
  return 0;
}

/* ------------------------------------------------------------------ apply_delete (transaction.rs:472-578) */
/* applies ds (hb order); the unapplied part goes to (un, unv) */
static void t_apply_delete(sdoc_t *d, const hb_t *ds, const idr_t *dsv, hb_t *un, idrvec_t *unv) {
  int32_t *ord = malloc((ds->items + 1) * sizeof(int32_t));
  size_t k = hb_order(ds, ord);
  for (size_t q = 0; q < k && !d->err; q++) {
    uint64_t client = ds->keys.d[ord[q]];
    const idr_t *g = &dsv[ord[q]];
    slist_t *l = s_list(d, client);
    if (!l) continue;
    uint32_t state = s_clock(d, client);
    size_t nr = g->cont ? 1 : g->v.n;
    for (size_t ri = 0; ri < nr; ri++) {
      rng_t r = g->cont ? g->c : g->v.d[ri];
      uint32_t clock = r.s, clock_end = r.e;
      if (clock >= state) {
        idset_insert(un, unv, client, clock, clock_end - clock);
        continue;
      }
      if (state < clock_end) idset_insert(un, unv, client, state, clock_end - state);
      l = s_list(d, client);
      int64_t idx = s_pivot(d, l, clock);
      if (idx < 0 || l->v.d[idx].gc) continue; /* GC / deleted structs are skipped */
      int32_t xi = l->v.d[idx].item;
      if (!d->it.d[xi].deleted && d->it.d[xi].clock < clock) {
        int32_t sp = s_split(d, xi, clock - d->it.d[xi].clock);
        if (sp >= 0) {
          idx++;
          sid_t id = {d->it.d[sp].client, d->it.d[sp].clock};
          VPUSH(d->merge_blocks, id);
        }
        l = s_list(d, client);
      }
      while ((size_t)idx < l->v.n && !d->err) {
        if (!l->v.d[idx].gc) {
          int32_t yi = l->v.d[idx].item;
          if (d->it.d[yi].clock >= clock_end) break;
          if (!d->it.d[yi].deleted) {
            if (d->it.d[yi].clock + d->it.d[yi].len > clock_end) {
              int32_t sp = s_split(d, yi, clock_end - d->it.d[yi].clock);
              if (sp >= 0) {
                sid_t id = {d->it.d[sp].client, d->it.d[sp].clock};
                VPUSH(d->merge_blocks, id);
                idx++;
              }
            }
            t_delete(d, yi);
            l = s_list(d, client);
          }
        }
        idx++;
      }
    }
  }
  free(ord);
}

/* ------------------------------------------------------------------ squash (block_store.rs, block.rs:775-799) */
static bool s_item_try_squash(sdoc_t *d, int32_t ai, int32_t bi) {
  sitem_t *a = &d->it.d[ai], *b = &d->it.d[bi];
  if (!(a->client == b->client && a->clock + a->len == b->clock && b->has_origin && b->oc == a->client &&
        b->ok == a->clock + a->len - 1 && s_same_ro(a, b) && a->right == bi && a->deleted == b->deleted))
    return false;
  if (!sc_try_squash(a, b)) return false;
  a->len = a->ref == 1 ? a->len : sc_len(a);
  if (b->right >= 0) d->it.d[b->right].left = ai;
  if (b->keep) a->keep = 1;
  a->right = b->right;
  return true;
}
static void s_fix_map(sdoc_t *d, int32_t ai, int32_t bi) {
  const sitem_t *b = &d->it.d[bi];
  if (b->has_psub && b->parent >= 0 && br_map_get(d, b->parent, b->psub) == bi) br_map_set(d, b->parent, b->psub, ai);
}
/* ClientBlockList::squash_left (block_store.rs:243-271) */
static void s_squash_left(sdoc_t *d, slist_t *l, size_t index) {
  cell_t *L = &l->v.d[index - 1], *R = &l->v.d[index];
  if (L->gc && R->gc) {
    L->end = R->end;
  } else if (!L->gc && !R->gc) {
    if (!s_item_try_squash(d, L->item, R->item)) return;
    s_fix_map(d, L->item, R->item);
  } else
    return;
  memmove(l->v.d + index, l->v.d + index + 1, (l->v.n - index - 1) * sizeof(cell_t));
  l->v.n--;
}
/* squash_left_range_compaction (block_store.rs:155-241) */
static void s_squash_range(sdoc_t *d, slist_t *l, size_t lo, size_t hi) {
  typedef struct {
    size_t s, e;
    int gc;
  } sq_t;
  VEC(sq_t) iv = {0};
  for (size_t ri = hi + 1; ri-- > lo;) {
    cell_t *L = &l->v.d[ri - 1], *R = &l->v.d[ri];
    if (L->gc && R->gc) {
      bool ext = false;
      if (iv.n && iv.d[iv.n - 1].gc && iv.d[iv.n - 1].s - 1 == ri) {
        iv.d[iv.n - 1].s = ri;
        ext = true;
      }
      if (!ext) {
        sq_t q = {ri, ri, 1};
        VPUSH(iv, q);
      }
    } else if (!L->gc && !R->gc) {
      if (s_item_try_squash(d, L->item, R->item)) {
        sq_t q = {ri, ri, 0};
        VPUSH(iv, q);
      }
    }
  }
  for (size_t q = 0; q < iv.n; q++) {
    size_t s = iv.d[q].s, e = iv.d[q].e;
    cell_t *L = &l->v.d[s - 1], *R = &l->v.d[e];
    if (L->gc && R->gc)
      L->end = R->end;
    else if (!L->gc && !R->gc)
      s_fix_map(d, L->item, R->item);
    memmove(l->v.d + s, l->v.d + e + 1, (l->v.n - e - 1) * sizeof(cell_t));
    l->v.n -= e - s + 1;
  }
  VFREE(iv);
}

/* ------------------------------------------------------------------ commit (transaction.rs:828-910) */
static void s_gc_item(sdoc_t *d, int32_t xi, bool parent_gc, sidvec_t *marks);
static void s_gc_content(sdoc_t *d, int32_t xi, sidvec_t *marks) { /* ItemContent::gc (block.rs:1907-1926) */
  sitem_t *x = &d->it.d[xi];
  if (x->ref != 7 || x->branch < 0) return;
  branch_t *B = &d->br.d[x->branch];
  int32_t cur = B->start;
  B->start = -1;
  while (cur >= 0) {
    int32_t nx = d->it.d[cur].right;
    s_gc_item(d, cur, true, marks);
    cur = nx;
  }
  B = &d->br.d[x->branch];
  for (size_t i = 0; i < B->vals.n; i++) {
    int32_t c2 = B->vals.d[i];
    while (c2 >= 0) {
      int32_t nx = d->it.d[c2].left;
      s_gc_item(d, c2, true, marks);
      c2 = nx;
    }
  }
  B = &d->br.d[x->branch];
  B->keys.n = 0;
  B->vals.n = 0;
}
static void s_gc_item(sdoc_t *d, int32_t xi, bool parent_gc, sidvec_t *marks) { /* Item::gc */
  sitem_t *x = &d->it.d[xi];
  if (x->deleted && !x->keep) {
    s_gc_content(d, xi, marks);
    x = &d->it.d[xi];
    if (parent_gc) {
      sid_t id = {x->client, x->clock};
      VPUSH(*marks, id);
    } else {
      VFREE(x->str);
      VFREE(x->el);
      x->ref = 1; /* ItemContent::Deleted(len) */
      x->countable = 0;
    }
  }
}
static void t_commit(sdoc_t *d) {
  /* 1. squash the delete set */
  for (size_t i = 0; i < d->tdsv.n; i++) idr_squash(&d->tdsv.d[i]);
  /* 4. GC (gc.rs:10-66): mark_all then collect_all_marked */
  sidvec_t marks = {0};
  int32_t *ord = malloc((d->tds.items + 1) * sizeof(int32_t));
  size_t k = hb_order(&d->tds, ord);
  for (size_t q = 0; q < k; q++) {
    uint64_t client = d->tds.keys.d[ord[q]];
    const idr_t *g = &d->tdsv.d[ord[q]];
    slist_t *l = s_list(d, client);
    if (!l) continue;
    size_t nr = g->cont ? 1 : g->v.n;
    for (size_t ri = nr; ri-- > 0;) {
      rng_t r = g->cont ? g->c : g->v.d[ri];
      uint32_t start = r.s;
      int64_t i = s_pivot(d, l, start);
      if (i < 0) continue;
      while ((size_t)i < l->v.n) {
        cell_t *c = &l->v.d[i];
        uint32_t len = c->gc ? c->end - c->start + 1 : d->it.d[c->item].len;
        start += len;
        if (start > r.e) break;
        if (!c->gc) s_gc_item(d, c->item, false, &marks);
        l = s_list(d, client);
        i++;
      }
    }
  }
  for (size_t m = 0; m < marks.n; m++) {
    slist_t *l = s_list_mut(d, marks.d[m].client);
    int64_t i = s_pivot(d, l, marks.d[m].clock);
    if (i < 0) continue;
    cell_t *c = &l->v.d[i];
    if (!c->gc && d->it.d[c->item].deleted && !d->it.d[c->item].keep) {
      uint32_t s = d->it.d[c->item].clock, e = s + d->it.d[c->item].len - 1;
      c->gc = 1;
      c->start = s;
      c->end = e;
    }
  }
  VFREE(marks);
  /* 5. DeleteSet::try_squash_with (id_set.rs:571-598) */
  for (size_t q = 0; q < k; q++) {
    uint64_t client = d->tds.keys.d[ord[q]];
    const idr_t *g = &d->tdsv.d[ord[q]];
    slist_t *l = s_list_mut(d, client);
    size_t nr = g->cont ? 1 : g->v.n;
    for (size_t ri = nr; ri-- > 0;) {
      rng_t r = g->cont ? g->c : g->v.d[ri];
      if (!l->v.n) break;
      int64_t p = s_pivot(d, l, r.e - 1);
      size_t si = l->v.n - 1 < (size_t)(1 + (p < 0 ? 0 : p)) ? l->v.n - 1 : (size_t)(1 + (p < 0 ? 0 : p));
      size_t vlo = SIZE_MAX, vhi = 0;
      while (si > 0 && cell_start(d, &l->v.d[si]) >= r.s) {
        if (si < vlo) vlo = si;
        if (si > vhi) vhi = si;
        si--;
      }
      if (vlo != SIZE_MAX) s_squash_range(d, l, vlo, vhi);
    }
  }
  free(ord);
  /* 6. squash the blocks added by the transaction with their left neighbours */
  for (size_t e = 0; e < d->clients.keys.n; e++) {
    uint64_t client = d->clients.keys.d[e];
    uint32_t after = s_clock(d, client);
    int32_t be = hb_find(&d->before, client);
    uint32_t before = be >= 0 ? d->before_clock.d[be] : 0;
    if (before == after) continue;
    slist_t *l = &d->lists.d[e];
    int64_t fc = s_pivot(d, l, before);
    if (fc < 0) fc = 0; /* (find_pivot on a new client's list) */
    size_t first = fc > 1 ? (size_t)fc : 1;
    for (size_t i = l->v.n - 1; i >= first && i > 0; i--) s_squash_left(d, l, i);
  }
  /* 7. merge_blocks */
  for (size_t m = 0; m < d->merge_blocks.n; m++) {
    slist_t *l = s_list(d, d->merge_blocks.d[m].client);
    if (!l) continue;
    int64_t p = s_pivot(d, l, d->merge_blocks.d[m].clock);
    if (p < 0) continue;
    if ((size_t)p + 1 < l->v.n)
      s_squash_left(d, l, (size_t)p + 1);
    else if (p > 0)
      s_squash_left(d, l, (size_t)p);
  }
}
static void t_begin(sdoc_t *d) {
  hb_free(&d->before);
  d->before_clock.n = 0;
  for (size_t e = 0; e < d->clients.keys.n; e++) {
    bool ex;
    hb_insert(&d->before, d->clients.keys.d[e], &ex);
    VPUSH(d->before_clock, s_clock(d, d->clients.keys.d[e]));
  }
  hb_free(&d->tds);
  for (size_t i = 0; i < d->tdsv.n; i++) idr_free(&d->tdsv.d[i]);
  d->tdsv.n = 0;
  d->merge_blocks.n = 0;
}

/* ------------------------------------------------------------------ Update::integrate (update.rs:169-308) */
typedef struct {
  uint64_t client;
  u32vec_t q; /* VecDeque<BlockCarrier>: block indices of the decoded update */
  size_t head;
  int present;     /* still in UpdateBlocks.clients (return_stack removes it) */
} uq_t;
typedef struct {
  uint64_t client;
  u32vec_t q;
} rq_t;
typedef VEC(rq_t) rqvec_t;

static uq_t *uq_get(uq_t *qs, size_t nq, uint64_t client) {
  for (size_t i = 0; i < nq; i++)
    if (qs[i].client == client && qs[i].present) return &qs[i];
  return NULL;
}
static bool uq_pop(uq_t *q, uint32_t *b) {
  if (!q || q->head >= q->q.n) return false;
  *b = q->q.d[q->head++];
  return true;
}
/* return_stack (update.rs:411-431) */
static void return_stack(u32vec_t *stack, const upd_t *u, uq_t *qs, size_t nq, rqvec_t *rem) {
  for (size_t i = 0; i < stack->n; i++) {
    uint32_t bi = stack->d[i];
    uint64_t client = u->blocks.d[bi].client;
    uq_t *q = uq_get(qs, nq, client);
    rq_t r;
    memset(&r, 0, sizeof(r));
    r.client = client;
    VPUSH(r.q, bi);
    if (q) {
      for (size_t k = q->head; k < q->q.n; k++) VPUSH(r.q, q->q.d[k]);
      q->present = 0;
    }
    /* remaining.clients.insert(client, ..): replaces a previous entry */
    bool put = false;
    for (size_t k = 0; k < rem->n; k++)
      if (rem->d[k].client == client) {
        VFREE(rem->d[k].q);
        rem->d[k] = r;
        put = true;
      }
    if (!put) VPUSH(*rem, r);
  }
  stack->n = 0;
}
/* StateVector get / set_min / set_max over (hb, clocks) */
static uint32_t svh_get(const hb_t *t, const u32vec_t *c, uint64_t client) {
  int32_t e = hb_find(t, client);
  return e >= 0 ? c->d[e] : 0;
}
static void svh_set_min(hb_t *t, u32vec_t *c, uint64_t client, uint32_t clock) {
  bool ex;
  int32_t e = hb_entry(t, client, &ex);
  if (!ex)
    VPUSH(*c, clock);
  else if (clock < c->d[e])
    c->d[e] = clock;
}
static void svh_set_max(hb_t *t, u32vec_t *c, uint64_t client, uint32_t clock) {
  bool ex;
  int32_t e = hb_entry(t, client, &ex);
  if (!ex)
    VPUSH(*c, clock);
  else if (clock > c->d[e])
    c->d[e] = clock;
}
/* Update::missing (update.rs:310-345) on a decoded (not yet repaired) block */
static bool blk_missing(const blk_t *b, const hb_t *sv, const u32vec_t *svc, uint64_t *dep) {
  if (b->kind != BK_ITEM) return false;
  if (b->has_origin && b->oc != b->client && b->ok >= svh_get(sv, svc, b->oc)) {
    *dep = b->oc;
    return true;
  }
  if (b->has_ro && b->rc != b->client && b->rk >= svh_get(sv, svc, b->rc)) {
    *dep = b->rc;
    return true;
  }
  if (b->pkind == PK_ID && b->pc != b->client && b->pk >= svh_get(sv, svc, b->pc)) {
    *dep = b->pc;
    return true;
  }
  return false;
}
static int cmp_u64_asc(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? -1 : x > y;
}

/* encodes remaining blocks + missing as the pending update bytes (Update::encode_v1 with an
 * empty delete set) */
static int encode_remaining(const upd_t *u, rqvec_t *rem, wb_t *w) {
  clist_t *cl = calloc(rem->n + 1, sizeof(clist_t));
  for (size_t i = 0; i < rem->n; i++) {
    cl[i].client = rem->d[i].client;
    for (size_t k = 0; k < rem->d[i].q.n; k++) {
      car_t c = car_of(&u->blocks.d[rem->d[i].q.d[k]]);
      VPUSH(cl[i].cars, c);
      VPUSH(cl[i].ups, u);
    }
  }
  int e = encode_blocks(w, cl, rem->n, NULL);
  wb_var(w, 0); /* empty delete set */
  for (size_t i = 0; i < rem->n; i++) {
    VFREE(cl[i].cars);
    VFREE(cl[i].ups);
  }
  free(cl);
  return e;
}

/* Update::integrate: returns the pending update (bytes, missing) and the unapplied DS */
static int s_update_integrate(sdoc_t *d, const upd_t *u, wb_t *pend, int *has_pend, hb_t *miss, u32vec_t *miss_c,
                              hb_t *un, idrvec_t *unv) {
  *has_pend = 0;
  size_t nq = u->clients.keys.n;
  uq_t *qs = calloc(nq + 1, sizeof(uq_t));
  uint64_t *ids = malloc((nq + 1) * sizeof(uint64_t));
  for (size_t e = 0; e < nq; e++) {
    qs[e].client = u->clients.keys.d[e];
    qs[e].present = 1;
    for (size_t k = 0; k < u->lists.d[e].idx.n; k++) VPUSH(qs[e].q, u->lists.d[e].idx.d[k]);
    ids[e] = qs[e].client;
  }
  qsort(ids, nq, sizeof(uint64_t), cmp_u64_asc);
  size_t nids = nq;
  rqvec_t rem = {0};
  u32vec_t stack = {0};
  int err = 0;
  if (nq) {
    uint64_t cur_client = ids[--nids];
    uq_t *cur = uq_get(qs, nq, cur_client);
    uint32_t head;
    bool has_head = uq_pop(cur, &head);
    /* local state vector: the store's */
    hb_t lsv = {0};
    u32vec_t lsvc = {0};
    for (size_t e = 0; e < d->clients.keys.n; e++) {
      bool ex;
      hb_insert(&lsv, d->clients.keys.d[e], &ex);
      VPUSH(lsvc, s_clock(d, d->clients.keys.d[e]));
    }
    while (has_head && !err && !d->err) {
      const blk_t *b = &u->blocks.d[head];
      if (b->kind != BK_SKIP) {
        uint32_t lc = svh_get(&lsv, &lsvc, b->client);
        if (b->clock <= lc) {
          uint32_t offset = lc - b->clock;
          uint64_t dep;
          if (blk_missing(b, &lsv, &lsvc, &dep)) {
            VPUSH(stack, head);
            uq_t *dq = uq_get(qs, nq, dep);
            if (dq && dq->head < dq->q.n) {
              uq_pop(dq, &head);
              cur = uq_get(qs, nq, cur_client);
              continue;
            }
            svh_set_min(miss, miss_c, dep, svh_get(&lsv, &lsvc, dep));
            return_stack(&stack, u, qs, nq, &rem);
            cur = uq_get(qs, nq, cur_client);
          } else if (offset == 0 || offset < b->len) {
            svh_set_max(&lsv, &lsvc, b->client, b->clock + b->len);
            if (b->kind == BK_GC) {
              slist_t *l = s_list_mut(d, b->client);
              cell_t c = {1, -1, b->clock + offset, b->clock + b->len - 1};
              VPUSH(l->v, c);
            } else {
              int32_t xi;
              err = s_item_from(d, u, b, &xi);
              if (err) break;
              s_repair(d, xi);
              if (d->err) break;
              int del = s_integrate(d, xi, offset);
              if (d->err) break;
              sitem_t *x = &d->it.d[xi];
              if (x->parent >= 0) {
                slist_t *l = s_list_mut(d, x->client);
                cell_t c = {0, xi, 0, 0};
                VPUSH(l->v, c);
                if (del) t_delete(d, xi);
              } else { /* parent unknown (GC'd): a GC struct instead */
                slist_t *l = s_list_mut(d, x->client);
                cell_t c = {1, -1, x->clock, x->clock + x->len - 1};
                VPUSH(l->v, c);
              }
            }
          }
        } else {
          svh_set_min(miss, miss_c, b->client, b->clock - 1);
          VPUSH(stack, head);
          return_stack(&stack, u, qs, nq, &rem);
          cur = uq_get(qs, nq, cur_client);
        }
      }
      /* next stack head */
      if (stack.n) {
        head = stack.d[--stack.n];
        has_head = true;
      } else if (cur && cur->head < cur->q.n) {
        uq_pop(cur, &head);
        has_head = true;
      } else {
        has_head = false;
        while (nids) {
          uint64_t id = ids[--nids];
          uq_t *q = uq_get(qs, nq, id);
          if (q && q->head < q->q.n) {
            cur_client = id;
            cur = q;
            uq_pop(cur, &head);
            has_head = true;
            break;
          }
        }
      }
    }
    hb_free(&lsv);
    VFREE(lsvc);
  }
  if (!err && !d->err && rem.n) {
    err = encode_remaining(u, &rem, pend);
    *has_pend = 1;
  }
  for (size_t i = 0; i < rem.n; i++) VFREE(rem.d[i].q);
  VFREE(rem);
  VFREE(stack);
  for (size_t e = 0; e < nq; e++) VFREE(qs[e].q);
  free(qs);
  free(ids);
  if (!err && !d->err) t_apply_delete(d, &u->ds, u->dsv.d, un, unv);
  return err ? err : d->err;
}

/* ------------------------------------------------------------------ apply_update (transaction.rs:664-726) */
static void ds_bytes(wb_t *w, const hb_t *t, const idr_t *v) { /* Update { blocks: [], delete_set } */
  wb_var(w, 0);
  ds_encode(w, t, v);
}
static int merge2(const uint8_t *a, size_t an, const uint8_t *b, size_t bn, uint8_t **out, size_t *on) {
  const uint8_t *p[2] = {a, b};
  size_t l[2] = {an, bn};
  return yo_merge_updates_v1(p, l, 2, 1, out, on);
}
static int s_apply_update(sdoc_t *d, const uint8_t *bytes, size_t n, int depth) {
  if (depth > 64) return YO_ERR_UNSUPPORTED;
  upd_t *u = calloc(1, sizeof(upd_t));
  /* the decoded blocks point into `bytes`: keep a copy alive for the document's lifetime */
  uint8_t *own = malloc(n + 1);
  memcpy(own, bytes, n);
  VPUSH(d->owned, own);
  int err = decode_update(u, own, n);
  if (!err && u->unsupported) err = YO_ERR_UNSUPPORTED;
  wb_t pend = {0};
  int has_pend = 0;
  hb_t miss = {0};
  u32vec_t missc = {0};
  hb_t un = {0};
  idrvec_t unv = {0};
  if (!err) err = s_update_integrate(d, u, &pend, &has_pend, &miss, &missc, &un, &unv);
  bool retry = false;
  if (!err) {
    if (d->has_pend) {
      for (size_t e = 0; e < d->pmiss.keys.n; e++)
        if (d->pmiss_clock.d[e] < s_clock(d, d->pmiss.keys.d[e])) {
          retry = true;
          break;
        }
      if (has_pend) {
        for (size_t e = 0; e < miss.keys.n; e++)
          svh_set_min(&d->pmiss, &d->pmiss_clock, miss.keys.d[e], missc.d[e]);
        uint8_t *m;
        size_t mn;
        err = merge2(d->pend.d, d->pend.n, pend.d, pend.n, &m, &mn);
        if (!err) {
          d->pend.n = 0;
          for (size_t i = 0; i < mn; i++) VPUSH(d->pend, m[i]);
          free(m);
        }
      }
    } else if (has_pend) {
      d->has_pend = 1;
      d->pend.n = 0;
      for (size_t i = 0; i < pend.n; i++) VPUSH(d->pend, pend.d[i]);
      hb_free(&d->pmiss);
      d->pmiss_clock.n = 0;
      for (size_t e = 0; e < miss.keys.n; e++) {
        bool ex;
        hb_insert(&d->pmiss, miss.keys.d[e], &ex);
        VPUSH(d->pmiss_clock, missc.d[e]);
      }
    }
  }
  if (!err) {
    /* pending delete set: re-apply it, keep what is still unapplied (merged with this update's) */
    if (d->has_pend_ds) {
      upd_t pu;
      int e2 = decode_update(&pu, d->pend_ds.d, d->pend_ds.n);
      hb_t un2 = {0};
      idrvec_t unv2 = {0};
      if (!e2) t_apply_delete(d, &pu.ds, pu.dsv.d, &un2, &unv2);
      /* (Some(a), Some(b)) => a.merge(b): IdSet::merge (id_set.rs:381-390) */
      hb_t *rt = &un;
      idrvec_t *rv = &unv;
      if (un.items && un2.items) {
        int32_t *ord = malloc((un2.items + 1) * sizeof(int32_t));
        size_t k = hb_order(&un2, ord);
        for (size_t q = 0; q < k; q++) {
          bool ex;
          int32_t e = hb_insert(&un, un2.keys.d[ord[q]], &ex);
          if (ex)
            idr_merge(&unv.d[e], &unv2.d[ord[q]]);
          else {
            idr_t c;
            idr_clone(&c, &unv2.d[ord[q]]);
            VPUSH(unv, c);
          }
        }
        free(ord);
        for (size_t q = 0; q < unv.n; q++) idr_squash(&unv.d[q]);
      } else if (!un.items && un2.items) {
        rt = &un2;
        rv = &unv2;
      }
      d->pend_ds.n = 0;
      d->has_pend_ds = rt->items > 0;
      if (d->has_pend_ds) {
        wb_t w = {0};
        ds_bytes(&w, rt, rv->d);
        for (size_t i = 0; i < w.n; i++) VPUSH(d->pend_ds, w.d[i]);
        VFREE(w);
      }
      for (size_t q = 0; q < unv2.n; q++) idr_free(&unv2.d[q]);
      VFREE(unv2);
      hb_free(&un2);
      if (!e2) upd_free(&pu);
    } else {
      d->has_pend_ds = un.items > 0;
      d->pend_ds.n = 0;
      if (d->has_pend_ds) {
        wb_t w = {0};
        ds_bytes(&w, &un, unv.d);
        for (size_t i = 0; i < w.n; i++) VPUSH(d->pend_ds, w.d[i]);
        VFREE(w);
      }
    }
  }
  VFREE(pend);
  hb_free(&miss);
  VFREE(missc);
  for (size_t q = 0; q < unv.n; q++) idr_free(&unv.d[q]);
  VFREE(unv);
  hb_free(&un);
  upd_free(u);
  free(u);
  if (!err && retry && d->has_pend) {
    VEC(uint8_t) p = {0};
    VEC(uint8_t) pds = {0};
    for (size_t i = 0; i < d->pend.n; i++) VPUSH(p, d->pend.d[i]);
    if (d->has_pend_ds)
      for (size_t i = 0; i < d->pend_ds.n; i++) VPUSH(pds, d->pend_ds.d[i]);
    else {
      VPUSH(pds, 0);
      VPUSH(pds, 0);
    }
    d->has_pend = 0;
    d->pend.n = 0;
    d->has_pend_ds = 0;
    d->pend_ds.n = 0;
    hb_free(&d->pmiss);
    d->pmiss_clock.n = 0;
    err = s_apply_update(d, p.d, p.n, depth + 1);
    if (!err) err = s_apply_update(d, pds.d, pds.n, depth + 1);
    VFREE(p);
    VFREE(pds);
  }
  return err;
}

/* ------------------------------------------------------------------ encode_state_as_update_v1 */
static int s_encode_content(wb_t *w, const sdoc_t *d, const sitem_t *x) {
  switch (x->ref) {
  case 1: wb_var(w, x->len); return 0;
  case 2:
    wb_var(w, (uint32_t)x->el.n);
    for (size_t i = 0; i < x->el.n; i++) wb_str(w, x->el.d[i].p, x->el.d[i].n);
    return 0;
  case 3: wb_str(w, x->cs.p, x->cs.n); return 0;
  case 4: wb_str(w, x->str.d, (uint32_t)x->str.n); return 0;
  case 5: case 6: {
    if (x->ref == 6) wb_str(w, x->cs.p, x->cs.n);
    const span_t js = x->ref == 6 ? x->cs2 : x->cs;
    wb_t t = {0};
    int e = json_canon(js.p, js.n, &t);
    if (!e) wb_str(w, t.d, (uint32_t)t.n);
    VFREE(t);
    return e;
  }
  case 7:
    wb_u8(w, x->tref);
    if (x->tref == 3) wb_str(w, x->cs.p, x->cs.n);
    return 0;
  case 8:
    wb_var(w, (uint32_t)x->el.n);
    for (size_t i = 0; i < x->el.n; i++) {
      rd_t r = {x->el.d[i].p, x->el.d[i].n, 0};
      any_encode(&r, w);
    }
    return 0;
  }
  return YO_ERR_REFERENCE_PANIC;
}
/* Item encode (block.rs:1363-1369 info; slice.rs:199-251 with no offset) */
static int s_encode_item(wb_t *w, const sdoc_t *d, const sitem_t *x) {
  uint8_t info = (x->has_origin ? 0x80 : 0) | (x->has_ro ? 0x40 : 0) | (x->has_psub ? 0x20 : 0) | (x->ref & 15);
  wb_u8(w, info);
  if (x->has_origin) {
    wb_var(w, x->oc);
    wb_var(w, x->ok);
  }
  if (x->has_ro) {
    wb_var(w, x->rc);
    wb_var(w, x->rk);
  }
  if (!x->has_origin && !x->has_ro) {
    if (x->parent < 0) return YO_ERR_REFERENCE_PANIC;
    const branch_t *B = &d->br.d[x->parent];
    if (B->item >= 0) {
      wb_var(w, 0);
      wb_var(w, d->it.d[B->item].client);
      wb_var(w, d->it.d[B->item].clock);
    } else {
      wb_var(w, 1);
      wb_str(w, B->name.p, B->name.n);
    }
    if (x->has_psub) wb_str(w, x->psub.p, x->psub.n);
  }
  return s_encode_content(w, d, x);
}
static int s_encode_state(sdoc_t *d, wb_t *w) {
  /* write_blocks_from(empty SV) (store.rs:204-232): clients with blocks, descending */
  size_t nc = d->clients.keys.n;
  uint64_t *cl = malloc((nc + 1) * sizeof(uint64_t));
  size_t k = 0;
  for (size_t e = 0; e < nc; e++)
    if (d->lists.d[e].v.n) cl[k++] = d->clients.keys.d[e];
  qsort(cl, k, sizeof(uint64_t), cmp_u64_desc);
  wb_var(w, k);
  for (size_t i = 0; i < k; i++) {
    slist_t *l = s_list(d, cl[i]);
    wb_var(w, l->v.n);
    wb_var(w, cl[i]);
    wb_var(w, cell_start(d, &l->v.d[0]));
    for (size_t j = 0; j < l->v.n; j++) {
      const cell_t *c = &l->v.d[j];
      if (c->gc) {
        wb_u8(w, 0);
        wb_var(w, c->end - c->start + 1);
      } else {
        int e = s_encode_item(w, d, &d->it.d[c->item]);
        if (e) {
          free(cl);
          return e;
        }
      }
    }
  }
  free(cl);
  /* DeleteSet::from(&BlockStore) (id_set.rs:448-468): store iteration order, IdRange::push */
  hb_t ds = {0};
  idrvec_t dv = {0};
  int32_t *ord = malloc((nc + 1) * sizeof(int32_t));
  size_t no = hb_order(&d->clients, ord);
  for (size_t q = 0; q < no; q++) {
    slist_t *l = &d->lists.d[ord[q]];
    idr_t g;
    memset(&g, 0, sizeof(g)); /* IdRange::with_capacity: Fragmented(empty) */
    for (size_t j = 0; j < l->v.n; j++)
      if (cell_deleted(d, &l->v.d[j])) {
        rng_t r = {cell_start(d, &l->v.d[j]), cell_end(d, &l->v.d[j]) + 1};
        idr_push(&g, r);
      }
    if (g.cont || g.v.n) {
      bool ex;
      int32_t e = hb_insert(&ds, d->clients.keys.d[ord[q]], &ex);
      if (ex) {
        idr_free(&dv.d[e]);
        dv.d[e] = g;
      } else
        VPUSH(dv, g);
    } else
      idr_free(&g);
  }
  free(ord);
  ds_encode(w, &ds, dv.d);
  for (size_t q = 0; q < dv.n; q++) idr_free(&dv.d[q]);
  VFREE(dv);
  hb_free(&ds);
  return 0;
}

static void s_free(sdoc_t *d) {
  for (size_t i = 0; i < d->it.n; i++) {
    VFREE(d->it.d[i].str);
    VFREE(d->it.d[i].el);
  }
  VFREE(d->it);
  hb_free(&d->clients);
  for (size_t i = 0; i < d->lists.n; i++) VFREE(d->lists.d[i].v);
  VFREE(d->lists);
  for (size_t i = 0; i < d->br.n; i++) {
    VFREE(d->br.d[i].keys);
    VFREE(d->br.d[i].vals);
  }
  VFREE(d->br);
  VFREE(d->pend);
  hb_free(&d->pmiss);
  VFREE(d->pmiss_clock);
  VFREE(d->pend_ds);
  for (size_t i = 0; i < d->owned.n; i++) free(d->owned.d[i]);
  VFREE(d->owned);
  hb_free(&d->before);
  VFREE(d->before_clock);
  hb_free(&d->tds);
  for (size_t i = 0; i < d->tdsv.n; i++) idr_free(&d->tdsv.d[i]);
  VFREE(d->tdsv);
  VFREE(d->merge_blocks);
}

/* Doc::new (GC on) -> for each update: transact_mut + apply_update + commit ->
 * encode_state_as_update_v1(&StateVector::default()) with the pending data merged in */
int yo_compact_updates_v1(const uint8_t *const *updates, const size_t *lens, size_t n, uint8_t **out,
                          size_t *out_len) {
  *out = NULL;
  *out_len = 0;
  sdoc_t d;
  memset(&d, 0, sizeof(d));
  int err = 0;
  for (size_t i = 0; i < n && !err; i++) {
    t_begin(&d);
    err = s_apply_update(&d, updates[i], lens[i], 0);
    if (!err) t_commit(&d);
    if (!err) err = d.err;
  }
  wb_t w = {0};
  if (!err) err = s_encode_state(&d, &w);
  if (!err && (d.has_pend || d.has_pend_ds)) { /* merge_pending_v1 (transaction.rs:247-263) */
    const uint8_t *p[3];
    size_t l[3], k = 0;
    p[k] = w.d ? w.d : (const uint8_t *)"";
    l[k++] = w.n;
    if (d.has_pend) {
      p[k] = d.pend.d;
      l[k++] = d.pend.n;
    }
    if (d.has_pend_ds) {
      p[k] = d.pend_ds.d;
      l[k++] = d.pend_ds.n;
    }
    uint8_t *m;
    size_t mn;
    err = yo_merge_updates_v1(p, l, k, 1, &m, &mn);
    if (!err) {
      VFREE(w);
      w.d = m;
      w.n = mn;
      w.cap = mn;
    }
  }
  s_free(&d);
  if (err) {
    free(w.d);
    return err;
  }
  return finish(&w, out, out_len);
}
