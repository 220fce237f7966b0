"""GPU parity on the reference's own corpora and on rich-text content.

* assets/bench-input/small-test-dataset.bin (5,320 real Yjs documents, 46,385 updates with
  Format/Embed/Type/Any content; tests/golden/small-test-dataset.bin): merge_updates_v1 of
  every document, status 0 and GPU == oracle byte for byte, on the fast path and on the
  exact engine; state vectors and diffs of the merged documents.
* ContentEmbed / ContentFormat JSON (serde_json + ryu restatement, tests/test_json.py) and
  Any maps with repeated keys, through the device codec.
"""
import os

import numpy as np
import pytest

import corpus
from test_gpu_parity import batch_of, check_batch
from test_json import SERDE_VECTORS, _content_update

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    import ymerge
    e = ymerge.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def dataset():
    return batch_of([d[0] for d in corpus.small_dataset()])


def test_small_dataset_merge(engine, oracle, dataset):
    out, off, st = check_batch(engine, oracle, dataset)
    assert not st.any()
    s = engine.stats()
    print(f"fast {s['docs_fast']} exact {s['docs_exact']}")


# Routing of the 5,320 corpus documents (round 5): k_lean takes the editor-shaped ones, the
# workgroup fast path the rich-content ones, the tiled kernel the 18 above the fast path's LDS
# capacities; none needs the exact engine (the tiny-document hand-over serves only batches of
# >= 262,144 documents) or the grid paths.  Update with the routing when it changes on purpose.
CORPUS_PATHS = {"docs_lean": 1385, "docs_fast": 3917, "docs_big": 18, "docs_exact": 0, "docs_tiny": 0,
                "docs_giant": 0, "docs_error": 0}


def test_small_dataset_paths(engine, oracle, dataset):
    """Per-path document counts on the reference corpus (bit-exact output checked as well)."""
    out, off, st = check_batch(engine, oracle, dataset)
    s = engine.stats()
    got = {k: int(s[k]) for k in CORPUS_PATHS}
    assert got == CORPUS_PATHS, got
    assert sum(got[k] for k in ("docs_lean", "docs_fast", "docs_big", "docs_exact", "docs_giant")) == dataset.n_docs


@pytest.mark.parametrize("env", [
    {"YMERGE_EXACT_LOCKSTEP": "1"},                            # exact decode one update per wavefront
    {"YMERGE_LP_MID": "100000", "YMERGE_EXACT_LOCKSTEP": "1"},  # rich updates on the exact walk only
    {"YMERGE_LP_MID": "16"},                                   # nearly every rich update on the parallel parse
    {"YMERGE_LONG_PARSE": "0"},                                # no parallel parse: the lockstep walker
    {"YMERGE_TINY": "4"},                                      # tiny documents on the exact engine's lanes
    {"YMERGE_LEAN_SPIN": "0"},  # k_lean's sharded hand-over count read by a copy, not the mapped signal
])
def test_small_dataset_decode_routes(oracle, dataset, env):
    """The corpus through every decode route the knobs select: the same bytes each time."""
    from test_gpu_parity import engine_with
    e = engine_with(**env)
    try:
        out, off, st = check_batch(e, oracle, dataset)
        assert not st.any()
    finally:
        e.close()


def test_small_dataset_exact_engine(oracle, dataset):
    import ymerge
    os.environ["YMERGE_FAST_THREADS"] = "0"
    try:
        e = ymerge.Engine(0)
    finally:
        del os.environ["YMERGE_FAST_THREADS"]
    try:
        check_batch(e, oracle, dataset)
    finally:
        e.close()


def test_small_dataset_sv_and_diff(engine, oracle, dataset):
    import workloads
    m, off, st = oracle.merge_batch(dataset.data, dataset.upd_off, dataset.doc_upd, mode=1, threads=8)
    m = np.frombuffer(m, np.uint8)
    sv, sv_off, sv_st = engine.state_vector_host(m, off)
    esv, esv_off, esv_st = oracle.sv_batch(m, off, threads=8)
    assert np.array_equal(sv_st, esv_st) and not sv_st.any()
    assert sv.tobytes() == esv and np.array_equal(sv_off, esv_off)
    rsv, rsv_off = workloads.remote_svs(np.frombuffer(esv, np.uint8), esv_off)
    df, df_off, df_st = engine.diff_host(m, off, rsv, rsv_off)
    edf, edf_off, edf_st = oracle.diff_batch(m, off, rsv, rsv_off, threads=8)
    assert np.array_equal(df_st, edf_st) and df.tobytes() == edf and np.array_equal(df_off, edf_off)


def _json_docs():
    docs = []
    for k, (src, _) in enumerate(SERDE_VECTORS):
        b = src.encode("latin-1") if "\xff" in src else src.encode()
        docs.append([_content_update(3 + k, 5, [b])])
        docs.append([_content_update(3 + k, 6, [b"attr", b]), _content_update(1000 + k, 4, [b"x"])])
    docs.append([_content_update(1, 5, [b"[" * 127 + b"]" * 127])])
    docs.append([_content_update(1, 5, [b"[" * 128 + b"]" * 128])])
    docs.append([_content_update(1, 6, [b"k", b'{"a":1e-320,"b":-1.7976931348623157e308,"c":[0.1,2.5e-8]}'])])
    return docs


def test_json_content_vectors(engine, oracle):
    check_batch(engine, oracle, batch_of(_json_docs()))


def test_json_content_exact_engine_and_sv(oracle):
    import ymerge
    os.environ["YMERGE_FAST_THREADS"] = "0"
    try:
        e = ymerge.Engine(0)
    finally:
        del os.environ["YMERGE_FAST_THREADS"]
    try:
        b = batch_of(_json_docs())
        check_batch(e, oracle, b)
        ups = [d[0] for d in _json_docs()]
        data = np.frombuffer(b"".join(ups), np.uint8)
        offs = np.concatenate([[0], np.cumsum([len(u) for u in ups])]).astype(np.uint64)
        sv, sv_off, st = e.state_vector_host(data, offs)
        esv, esv_off, est = oracle.sv_batch(data, offs, threads=4)
        assert np.array_equal(st, est) and sv.tobytes() == esv
    finally:
        e.close()


def test_any_map_duplicate_keys(engine, oracle):
    def s(b):
        return bytes([len(b)]) + b
    maps = [
        bytes([118, 3]) + s(b"a") + bytes([125, 1]) + s(b"b") + bytes([120]) + s(b"a") + bytes([125, 2]),
        bytes([118, 2]) + s(b"a") + bytes([118, 2]) + s(b"x") + bytes([126]) + s(b"x") + bytes([121])
        + s(b"a") + bytes([117, 1, 125, 5]),
        bytes([118, 4]) + s(b"k") + bytes([119]) + s(b"v1") + s(b"k") + bytes([119]) + s(b"v2") + s(b"j")
        + bytes([126]) + s(b"k") + bytes([120]),
    ]
    docs = [[bytes([1, 1, 9 + k, 0, 0x08, 1]) + s(b"map") + bytes([1]) + m + bytes([0])] for k, m in enumerate(maps)]
    check_batch(engine, oracle, batch_of(docs))
