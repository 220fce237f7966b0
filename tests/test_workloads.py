"""Synthetic workload generator: well-formed v1 updates the oracle accepts, shapes
as BASELINE.json describes."""
import numpy as np

import workloads


def test_c2_shape_and_validity(oracle):
    b = workloads.text_docs(40, 300)
    assert b.n_docs == 40 and b.n_updates == 40 * 300
    arena, off, st = oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=4)
    assert (st == 0).all()
    ratio = len(arena) / b.n_bytes
    assert 0.4 < ratio < 0.9


def test_deterministic():
    a = workloads.text_docs(5, 50)
    b = workloads.text_docs(5, 50)
    assert np.array_equal(a.data, b.data)


def test_c4_exercises_overlaps(oracle):
    b = workloads.delete_heavy_docs(4, ops_per_doc=600)
    arena, off, st = oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=0, threads=4)
    assert (st == 0).all()
    arena1, _, _ = oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=4)
    assert arena == arena1


def test_zipf_mean():
    k = workloads.zipf_counts(200_000)
    assert 60 < k.mean() < 95 and k.min() >= 1 and k.max() <= 10_000


def test_corpus_workloads_match_reference_readers():
    """bench.py --workload corpus: dataset_docs() reads every update of small-test-dataset.bin
    exactly as the test reader does (compatibility_tests.rs:437-476), tile() repeats documents
    in order, and traces' per-document update lists are the C1 replays."""
    import numpy as np
    import corpus
    import workloads
    ds = workloads.dataset_docs()
    ref = corpus.small_dataset()
    assert ds.n_docs == len(ref) == 5320
    for d in (0, 1, 77, 2600, 5319):
        assert ds.doc_updates(d) == [bytes(u) for u in ref[d][0]]
    t = workloads.tile(ds, 2 * ds.n_docs + 7)
    assert t.n_docs == 2 * ds.n_docs + 7
    for d in (0, 5, ds.n_docs + 5, 2 * ds.n_docs + 6):
        assert t.doc_updates(d) == ds.doc_updates(d % ds.n_docs)
    assert int(t.upd_off[-1]) == t.n_bytes and np.all(np.diff(t.upd_off.astype(np.int64)) >= 0)
