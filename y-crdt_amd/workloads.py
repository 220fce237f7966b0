"""Synthetic Yjs v1 update logs for the BASELINE.json configs (wraps csrc/workload.c).

C1  automerge-paper trace replay, one doc (tests/golden/automerge-paper.json.gz)
C2  n docs x k ops, 1-4 clients, 80/20 insert/delete, synced replicas (seed 0xC0FFEE)
C3  Zipf(1.5) op counts on [1, 1e4] (seed 0x5EED)
C4  delete-heavy docs: GC'd snapshot + per-op log, 10% withheld, 5% duplicated (seed 0xDE1E7E)
corpus  the reference's own inputs: assets/bench-input/small-test-dataset.bin (5,320 real Yjs
        documents, compatibility_tests.rs:437-476) tiled to a batch size, and the five
        assets/editing-traces sequential traces, one document each
"""
import ctypes
import functools
import gzip
import json
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "lib", "libywork.so")
_lib = None


def _L():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            raise RuntimeError(f"workload generator not built: {_LIB}")
        L = ctypes.CDLL(_LIB)
        P = ctypes.POINTER
        L.yw_generate.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32,
                                  ctypes.c_uint32, ctypes.c_double, ctypes.c_int, P(ctypes.c_void_p),
                                  P(ctypes.c_uint64), P(ctypes.c_void_p), P(ctypes.c_uint64), P(ctypes.c_void_p)]
        L.yw_replay.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_size_t,
                                ctypes.c_uint32, P(ctypes.c_void_p), P(ctypes.c_uint64), P(ctypes.c_void_p)]
        L.yw_generate_ids.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double, ctypes.c_int,
                                      P(ctypes.c_void_p), P(ctypes.c_uint64), P(ctypes.c_void_p), P(ctypes.c_uint64),
                                      P(ctypes.c_void_p)]
        L.yw_doc_hash.restype = ctypes.c_uint64
        L.yw_doc_hash.argtypes = [ctypes.c_uint64]
        L.yw_free.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


class Batch:
    """Arena of documents: doc d -> updates [doc_upd[d], doc_upd[d+1]) -> bytes [upd_off[u], upd_off[u+1])."""

    def __init__(self, data, upd_off, doc_upd, name=""):
        self.data, self.upd_off, self.doc_upd, self.name = data, upd_off, doc_upd, name

    @property
    def n_docs(self):
        return len(self.doc_upd) - 1

    @property
    def n_updates(self):
        return len(self.upd_off) - 1

    @property
    def n_bytes(self):
        return int(self.upd_off[-1])

    def doc_updates(self, d):
        u0, u1 = int(self.doc_upd[d]), int(self.doc_upd[d + 1])
        return [self.data[int(self.upd_off[u]):int(self.upd_off[u + 1])].tobytes() for u in range(u0, u1)]

    def prefix(self, n):
        """The first n documents (views into the same arena; offsets start at 0)."""
        u1 = int(self.doc_upd[n])
        return Batch(self.data[:int(self.upd_off[u1])], self.upd_off[:u1 + 1], self.doc_upd[:n + 1],
                     self.name + f"[:{n}]")

    def subset(self, docs):
        docs = list(docs)
        parts, offs, dus = [], [0], [0]
        tot = 0
        for d in docs:
            for u in self.doc_updates(d):
                parts.append(np.frombuffer(u, dtype=np.uint8))
                tot += len(u)
                offs.append(tot)
            dus.append(len(offs) - 1)
        data = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        return Batch(data, np.array(offs, np.uint64), np.array(dus, np.uint64), self.name + "[subset]")


def doc_hash(doc_id):
    return int(_L().yw_doc_hash(int(doc_id)))


def shard_ids(n_total, rank, world):
    """Global doc ids owned by `rank` under doc-hash sharding: splitmix64(id) % world == rank."""
    if world == 1:
        return np.arange(n_total, dtype=np.uint64)
    return np.array([i for i in range(n_total) if doc_hash(i) % world == rank], dtype=np.uint64)


def _generate(kind, seed, n_ops, min_clients, max_clients, del_frac, threads, ids=None):
    n_ops = np.ascontiguousarray(n_ops, dtype=np.uint32)
    b, nb, uo, nu, du = (ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_void_p(), ctypes.c_uint64(),
                         ctypes.c_void_p())
    idp = None
    if ids is not None:
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        assert len(ids) == len(n_ops)
        idp = ids.ctypes.data
    _L().yw_generate_ids(kind, seed, len(n_ops), idp, n_ops.ctypes.data, min_clients, max_clients, del_frac,
                         threads, ctypes.byref(b), ctypes.byref(nb), ctypes.byref(uo), ctypes.byref(nu),
                         ctypes.byref(du))
    data = np.frombuffer(ctypes.string_at(b, nb.value), dtype=np.uint8).copy() if nb.value else np.zeros(0, np.uint8)
    upd_off = np.ctypeslib.as_array(ctypes.cast(uo, ctypes.POINTER(ctypes.c_uint64)), (nu.value + 1,)).copy()
    doc_upd = np.ctypeslib.as_array(ctypes.cast(du, ctypes.POINTER(ctypes.c_uint64)), (len(n_ops) + 1,)).copy()
    for p in (b, uo, du):
        _L().yw_free(p)
    return data, upd_off, doc_upd


def text_docs(n_docs, ops_per_doc, seed=0xC0FFEE, min_clients=1, max_clients=4, del_frac=0.2, threads=None,
              ids=None):
    """C2: n_docs synced YText docs, `ops_per_doc` single-op updates each (ids: global doc ids)."""
    threads = threads or min(16, os.cpu_count() or 1)
    if ids is not None:
        n_docs = len(ids)
    n_ops = np.full(n_docs, ops_per_doc, np.uint32) if np.isscalar(ops_per_doc) else ops_per_doc
    return Batch(*_generate(2, seed, n_ops, min_clients, max_clients, del_frac, threads, ids), name="C2")


def zipf_counts(n_docs, alpha=1.5, kmax=10_000, seed=0x5EED):
    rng = np.random.default_rng(seed)
    k = np.arange(1, kmax + 1, dtype=np.float64)
    p = k ** (-alpha)
    cdf = np.cumsum(p / p.sum())
    return (np.searchsorted(cdf, rng.random(n_docs)) + 1).astype(np.uint32)


def zipf_docs(n_docs, seed=0x5EED, threads=None, ids=None):
    """C3: Zipf(1.5)-skewed update counts on [1, 1e4].  With `ids` (global doc ids of this
    shard) n_docs is the global document count and the shard's counts are drawn from it."""
    threads = threads or min(16, os.cpu_count() or 1)
    counts = zipf_counts(n_docs, seed=seed)
    if ids is not None:
        counts = counts[np.asarray(ids, dtype=np.int64)]
    return Batch(*_generate(2, seed, counts, 1, 4, 0.2, threads, ids), name="C3")


def delete_heavy_docs(n_docs, ops_per_doc=5000, seed=0xDE1E7E, threads=None):
    """C4: 70% deletes, GC'd snapshot + log with withheld / duplicated updates."""
    threads = threads or min(16, os.cpu_count() or 1)
    n_ops = np.full(n_docs, ops_per_doc, np.uint32)
    return Batch(*_generate(4, seed, n_ops, 1, 4, 0.7, threads), name="C4")


TRACES = ("automerge-paper", "friendsforever_flat", "rustcode", "seph-blog1", "sveltecomponent")


def trace_path(name):
    return os.path.join(os.path.dirname(_HERE), "tests", "golden", name + ".json.gz")


@functools.lru_cache(maxsize=8)
def trace_updates(path=None, client=1):
    """C1: one update per patch of an editing trace (default automerge-paper).

    Trace positions/lengths count Unicode scalar values; every trace here is BMP-only
    (checked below), so they equal the UTF-16 units yrs counts clocks in."""
    if path is None:
        path = trace_path("automerge-paper")
    elif not os.path.sep in path:
        path = trace_path(path)
    with gzip.open(path) as f:
        d = json.load(f)
    pos, dele, ilen, iun, ins = [], [], [], [], []
    for t in d["txns"]:
        for p in t["patches"]:
            if any(ord(c) > 0xFFFF for c in p[2]):
                raise ValueError("astral-plane text: trace positions would need UTF-16 remapping")
            s = p[2].encode("utf-8")
            pos.append(p[0])
            dele.append(p[1])
            ilen.append(len(s))
            iun.append(len(p[2]))
            ins.append(s)
    pos = np.array(pos, np.uint32)
    dele = np.array(dele, np.uint32)
    ilen = np.array(ilen, np.uint32)
    iun = np.array(iun, np.uint32)
    insb = np.frombuffer(b"".join(ins) or b"\0", dtype=np.uint8)
    b, nb, uo = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_void_p()
    _L().yw_replay(pos.ctypes.data, dele.ctypes.data, ilen.ctypes.data, iun.ctypes.data, insb.ctypes.data, len(pos),
                   client, ctypes.byref(b), ctypes.byref(nb), ctypes.byref(uo))
    data = np.frombuffer(ctypes.string_at(b, nb.value), dtype=np.uint8).copy()
    upd_off = np.ctypeslib.as_array(ctypes.cast(uo, ctypes.POINTER(ctypes.c_uint64)), (len(pos) + 1,)).copy()
    _L().yw_free(b)
    _L().yw_free(uo)
    return Batch(data, upd_off, np.array([0, len(pos)], np.uint64), name="C1"), d["endContent"]


def _golden(name):
    return os.path.join(os.path.dirname(_HERE), "tests", "golden", name)


@functools.lru_cache(maxsize=2)
def dataset_docs():
    """small-test-dataset.bin as a Batch of its 5,320 documents (each test's update list;
    the format test_data_set reads, yrs/src/tests/compatibility_tests.rs:437-476: var_u32
    count, per test var_u32 n + n read_buf updates, then the expected text / map / array,
    skipped here)."""
    data = open(_golden("small-test-dataset.bin"), "rb").read()
    n, i = _rv(data, 0)
    parts, offs, dus, tot = [], [0], [0], 0
    for _ in range(n):
        k, i = _rv(data, i)
        for _ in range(k):
            ln, i = _rv(data, i)
            parts.append(data[i:i + ln])
            tot += ln
            offs.append(tot)
            i += ln
        dus.append(len(offs) - 1)
        ln, i = _rv(data, i)  # expected text
        i += ln
        i = _skip_any(data, i)  # expected map
        i = _skip_any(data, i)  # expected array
    return Batch(np.frombuffer(b"".join(parts), np.uint8).copy(), np.array(offs, np.uint64),
                 np.array(dus, np.uint64), name="small-test-dataset")


def _skip_any(b, i):
    """Past one lib0 Any (yrs/src/any.rs:37-83)."""
    t = b[i]
    i += 1
    if t in (127, 126, 121, 120):
        return i
    if t == 125:  # signed varint
        while b[i] & 0x80:
            i += 1
        return i + 1
    if t in (124, 123, 122):
        return i + {124: 4, 123: 8, 122: 8}[t]
    if t in (119, 116):
        n, i = _rv(b, i)
        return i + n
    if t == 118:
        n, i = _rv(b, i)
        for _ in range(n):
            k, i = _rv(b, i)
            i = _skip_any(b, i + k)
        return i
    if t == 117:
        n, i = _rv(b, i)
        for _ in range(n):
            i = _skip_any(b, i)
        return i
    raise ValueError(f"bad Any tag {t}")


def tile(batch, n_docs):
    """The batch's documents repeated in order up to n_docs documents (one arena)."""
    reps = -(-n_docs // batch.n_docs)
    nb, nu = batch.n_bytes, batch.n_updates
    data = np.tile(batch.data[:nb], reps)
    uo = np.concatenate([batch.upd_off[:-1].astype(np.uint64) + np.uint64(r * nb) for r in range(reps)] +
                        [np.array([reps * nb], np.uint64)])
    du = np.concatenate([batch.doc_upd[:-1].astype(np.uint64) + np.uint64(r * nu) for r in range(reps)] +
                        [np.array([reps * nu], np.uint64)])
    full = Batch(data, uo, du, name=f"{batch.name}x{reps}")
    return full.prefix(n_docs) if n_docs < full.n_docs else full


def traces_batch():
    """The five sequential editing traces, one document each (per-op updates, client 1)."""
    bs = [trace_updates(t)[0] for t in TRACES]
    parts, uos, dus, tb, tu = [], [], [0], 0, 0
    for b in bs:
        parts.append(b.data[:b.n_bytes])
        uos.append(b.upd_off[:-1].astype(np.uint64) + np.uint64(tb))
        tb += b.n_bytes
        tu += b.n_updates
        dus.append(tu)
    return Batch(np.concatenate(parts), np.concatenate(uos + [np.array([tb], np.uint64)]),
                 np.array(dus, np.uint64), name="traces")


def _var(x):
    out = bytearray()
    while True:
        b, x = x & 0x7F, x >> 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _rv(b, i):
    v = s = 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        s += 7
        if x < 0x80:
            return v, i


def parse_sv(b):
    """Encoded state vector -> [(client, clock)] in stream order."""
    n, i = _rv(b, 0)
    out = []
    for _ in range(n):
        c, i = _rv(b, i)
        k, i = _rv(b, i)
        out.append((c, k))
    return out


def encode_sv(pairs):
    return _var(len(pairs)) + b"".join(_var(c) + _var(k) for c, k in pairs)


def remote_svs(sv_arena, sv_off, seed=0x5713):
    """C5 remote state vectors: per document, each client's remote clock drawn from
    {0, U[0, max), max - U[1, 8], max} (max = the document's own clock for that client).
    Returns (bytes, offsets)."""
    rng = np.random.default_rng(seed)
    parts, offs, tot = [], [0], 0
    for d in range(len(sv_off) - 1):
        own = parse_sv(bytes(sv_arena[int(sv_off[d]):int(sv_off[d + 1])]))
        pairs = []
        for c, mx in own:
            k = int(rng.integers(4))
            if k == 0:
                v = 0
            elif k == 1:
                v = int(rng.integers(0, max(1, mx)))
            elif k == 2:
                v = max(0, mx - int(rng.integers(1, 9)))
            else:
                v = mx
            pairs.append((c, v))
        rng.shuffle(pairs)
        e = encode_sv(pairs)
        parts.append(e)
        tot += len(e)
        offs.append(tot)
    return np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8)[:tot].copy(), np.array(offs, np.uint64)


class DiffBatch:
    """One update per document (+ one remote state vector per document for diff)."""

    def __init__(self, data, upd_off, sv=None, sv_off=None, name=""):
        self.data, self.upd_off, self.sv, self.sv_off, self.name = data, upd_off, sv, sv_off, name

    @property
    def n_docs(self):
        return len(self.upd_off) - 1

    @property
    def n_bytes(self):
        return int(self.upd_off[-1])

    def update(self, d):
        return self.data[int(self.upd_off[d]):int(self.upd_off[d + 1])].tobytes()


def compacted_docs(merged, offs, status=None, seed=0x5713, sv_fn=None):
    """C5 input from merged (compacted) documents: the merge outputs become the updates,
    remote state vectors are drawn against each document's own state vector (sv_fn:
    (data, off) -> (sv arena, sv offsets, status); the oracle or the engine)."""
    data = np.frombuffer(merged, dtype=np.uint8) if isinstance(merged, (bytes, bytearray)) else merged
    offs = np.asarray(offs, np.uint64)
    if status is not None and (np.asarray(status) != 0).any():
        keep = [d for d in range(len(offs) - 1) if status[d] == 0]
        parts = [data[int(offs[d]):int(offs[d + 1])] for d in keep]
        lens = np.array([len(p) for p in parts], np.uint64)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        data = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    sv, sv_off, st = sv_fn(data, offs)
    rsv, rsv_off = remote_svs(np.frombuffer(sv, np.uint8) if isinstance(sv, bytes) else sv, sv_off, seed)
    return DiffBatch(np.ascontiguousarray(data), offs, rsv, rsv_off, name="C5")
