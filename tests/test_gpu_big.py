"""GPU parity of the tiled kernel for documents above the fast path's LDS capacities
(ymerge_big.hip: > 1024 blocks, > 512 DeleteSet entries / ranges, > 64 distinct
DeleteSet clients) and the routing between the three device paths (fast, tiled, exact
engine).  Reference semantics: yrs/src/update.rs:537-704, yrs/src/id_set.rs:129-164."""
import numpy as np
import pytest

import workloads
from test_gpu_parity import _ds_update, _root_text_update, _var, batch_of, check_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    # k_lean off: every document here reaches the tiled kernel (or the exact engine) as it
    # would for shapes k_lean hands over (tests/test_gpu_lean.py covers k_lean's BIG mode)
    # (and the grid-wide long-document path off, so that C1 keeps exercising the tiled kernel;
    # tests/test_gpu_giant.py covers that path); the tiny-document route forced on (by default
    # it serves only batches of >= 262,144 documents handed to the fast path)
    from test_gpu_parity import engine_with
    e = engine_with(YMERGE_LEAN=0, YMERGE_GIANT_MIN=0, YMERGE_TINY=4)
    yield e
    e.close()


def test_c3_zipf_tail_on_tiled_kernel(engine, oracle):
    """C3 documents above 1024 blocks take the tiled kernel; none needs the exact engine."""
    b = workloads.zipf_docs(4000, seed=0x5EED)
    big = int((np.diff(b.doc_upd) > 1400).sum())  # > 1024 blocks (80% of the updates insert)
    assert big > 10
    check_batch(engine, oracle, b)
    st = engine.stats()
    assert st["docs_exact"] == 0, st
    assert st["docs_big"] >= big, st
    assert st["docs_tiny"] > 0, st  # documents of <= 4 updates: lane per document


def test_tiny_docs_on_fast_path(oracle):
    """The same Zipf documents with the tiny-document route off (YMERGE_TINY=0): the
    workgroup fast path must keep handling documents of 1-4 updates."""
    import os
    import ymerge
    os.environ["YMERGE_TINY"] = "0"
    try:
        e = ymerge.Engine(0)
    finally:
        del os.environ["YMERGE_TINY"]
    try:
        check_batch(e, oracle, workloads.zipf_docs(3000, seed=0x5EED + 1))
        st = e.stats()
        assert st["docs_tiny"] == 0 and st["docs_exact"] == 0, st
    finally:
        e.close()


def test_c1_trace_on_tiled_kernel(engine, oracle):
    """The whole automerge-paper trace (259,778 per-op updates, one document)."""
    b, _ = workloads.trace_updates()
    check_batch(engine, oracle, b)
    st = engine.stats()
    assert st["docs_big"] == 1 and st["docs_exact"] == 0, st


def test_large_multi_client_docs(engine, oracle):
    """Interleaved clients (the tiled kernel's stable sort) at several sizes around the
    2048-pair sort chunk and its merge passes."""
    docs = []
    for k, ops in enumerate((1100, 2047, 2049, 4100, 9000)):
        b = workloads.text_docs(2, ops, seed=100 + k, min_clients=3, max_clients=4)
        docs += [b.doc_updates(0), b.doc_updates(1)]
    check_batch(engine, oracle, batch_of(docs))
    assert engine.stats()["docs_exact"] == 0


def test_large_docs_client_counts(engine, oracle):
    """The tiled kernel's client counting sort (<= 8 clients) and its fallback to the
    general stable sort (9-12 clients), at 8 and 9 clients exactly and above."""
    docs = []
    for k, (lo, hi) in enumerate(((8, 8), (9, 9), (10, 12))):
        b = workloads.text_docs(2, 3000, seed=300 + k, min_clients=lo, max_clients=hi)
        docs += [b.doc_updates(0), b.doc_updates(1)]
    check_batch(engine, oracle, batch_of(docs))
    st = engine.stats()
    assert st["docs_exact"] == 0 and st["docs_big"] == 6, st


def test_shuffled_large_docs(engine, oracle):
    """Updates in random order (clock order restored by the sort), duplicated updates."""
    rng = np.random.default_rng(5)
    docs = []
    for n in (700, 1500, 3000):
        ups = []
        for c in (3, 9, 1 << 31):
            clock = 0
            for _ in range(n // 3):
                s = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, int(rng.integers(1, 5))))
                ups.append(_root_text_update(c, clock, s))
                clock += len(s)
        ups += [ups[int(i)] for i in rng.integers(0, len(ups), len(ups) // 10)]
        docs.append([ups[i] for i in rng.permutation(len(ups))])
    check_batch(engine, oracle, batch_of(docs))
    assert engine.stats()["docs_exact"] == 0


def test_big_deletesets(engine, oracle):
    """> 512 DeleteSet ranges / entries and > 64 distinct DeleteSet clients (tiled kernel's
    hash table, hashbrown order over up to 1024 clients, range sort and union)."""
    rng = np.random.default_rng(11)
    docs = []
    for n_cl, n_up, n_rng in ((3, 400, 3), (70, 80, 2), (300, 300, 1), (900, 1000, 1), (5, 2000, 4)):
        ups = []
        clients = [int(x) for x in rng.integers(0, 2 ** 32, n_cl)]
        for _ in range(n_up):
            ents = []
            for c in rng.choice(clients, size=min(3, n_cl), replace=False):
                rs = [(int(rng.integers(0, 5000)), int(rng.integers(1, 9))) for _ in range(n_rng)]
                ents.append((int(c), rs))
            ups.append(_ds_update(ents))
        ups.append(_root_text_update(7, 0, "hello"))
        docs.append(ups)
    check_batch(engine, oracle, batch_of(docs))
    st = engine.stats()
    assert st["docs_big"] >= 4, st


def test_big_doc_handovers(engine, oracle):
    """Big documents that must still leave the tiled kernel: a partial overlap (exact
    engine), a decode error in a late update (first error wins), > 1024 DeleteSet clients."""
    docs = []
    ups = [_root_text_update(5, i, "x") for i in range(1500)]
    ups.append(_root_text_update(5, 700, "abc"))  # [700, 703) partially overlaps 701/702
    docs.append(ups)
    ups = [_root_text_update(5, i, "y") for i in range(1500)]
    ups.insert(1400, b"\x01\x01")  # EndOfBuffer
    docs.append(ups)
    rng = np.random.default_rng(2)
    docs.append([_ds_update([(int(c), [(0, 1)])]) for c in rng.integers(0, 2 ** 32, 1100)])
    check_batch(engine, oracle, batch_of(docs))


def test_update_with_2p21_gc_blocks(engine, oracle):
    """One update of 2^21 + 5 GC blocks (4.2 MB), alone and twice (duplicate): above the
    decode record's 21-bit block count, through the lane clamp of the fast path's decode
    and on to the tiled kernel (ymerge_fast.hip hand-over); GPU == oracle."""
    from test_gpu_lean import var
    n = (1 << 21) + 5
    u = bytes([1]) + var(n) + var(77) + var(0) + bytes([0, 1]) * n + bytes([0])
    check_batch(engine, oracle, batch_of([[u], [u, u]]))


def test_document_of_2p23_updates(engine, oracle):
    """One document of 2^23 + 4 updates (2^23 + 3 empty ones around one insert): past the
    fast path's 23-bit update index (hand-over at U >= 2^23); GPU == oracle."""
    n = (1 << 23) + 3
    ins = np.frombuffer(bytes([1, 1, 5, 0, 4, 1, 1, ord("t"), 1, ord("a"), 0]), np.uint8)
    data = np.concatenate([np.tile(np.array([0, 0], np.uint8), n // 2), ins,
                           np.tile(np.array([0, 0], np.uint8), n - n // 2)])
    lens = np.full(n + 1, 2, np.uint64)
    lens[n // 2] = len(ins)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    b = workloads.Batch(data, off, np.array([0, n + 1], np.uint64))
    check_batch(engine, oracle, b)
