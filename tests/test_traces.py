"""The reference's editing traces (assets/editing-traces/sequential_traces, copied to
tests/golden/) replayed as one v1 update per patch (workloads.trace_updates).

Pinning (tools/yjs/check_traces.py, run in the build container): the oracle's
merge_updates_v1 of every trace, applied by the offline Yjs bundle, reproduces the trace's
endContent, and so does Yjs applying the merge of the first half of the updates followed
by diff_updates_v1(full merge, state vector of the half merge).  The fixture keeps the
sha256 of each of those results; the CPU tests re-derive them with the oracle, the GPU
tests with the engine."""
import hashlib
import json
import os

import numpy as np
import pytest

import workloads
from conftest import ROOT

FX = json.load(open(os.path.join(ROOT, "tests", "golden", "traces_yjs_check.json")))["results"]
FAST = ("friendsforever_flat", "rustcode", "seph-blog1", "sveltecomponent")


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def test_fixture_is_yjs_checked():
    assert set(FX) == set(workloads.TRACES)
    for name, r in FX.items():
        assert r["text_equal"] and r["diff_text_equal"], name


@pytest.mark.parametrize("name", FAST)
def test_oracle_trace(oracle, name):
    b, end = workloads.trace_updates(name)
    ups = b.doc_updates(0)
    assert len(ups) == FX[name]["updates"] and len(end) == FX[name]["end_len"]
    m = oracle.merge_updates_v1(ups, mode=1)
    assert sha(m) == FX[name]["merged_sha256"]
    half = oracle.merge_updates_v1(ups[: len(ups) // 2], mode=1)
    sv = oracle.encode_state_vector_from_update_v1(half)
    assert sha(half) == FX[name]["half_sha256"] and sha(sv) == FX[name]["sv_half_sha256"]
    assert sha(oracle.diff_updates_v1(m, sv)) == FX[name]["diff_sha256"]


def _arena(bufs):
    off = np.zeros(len(bufs) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in bufs])
    return np.frombuffer(b"".join(bufs), np.uint8), off


@pytest.mark.gpu
def test_gpu_traces(oracle):
    """All five traces in one batch (each a document above the fast path's capacities),
    then their first halves; SV and diff of the halves through the engine."""
    import ymerge
    e = ymerge.Engine(0)
    try:
        full, halves = [], []
        for name in workloads.TRACES:
            b, _ = workloads.trace_updates(name)
            ups = b.doc_updates(0)
            full.append(ups)
            halves.append(ups[: len(ups) // 2])
        from test_gpu_parity import batch_of
        res = []
        for docs in (full, halves):
            bt = batch_of(docs)
            out, off, st = e.merge_host(bt.data, bt.upd_off, bt.doc_upd)
            assert not st.any()
            res.append([out[int(off[d]):int(off[d + 1])].tobytes() for d in range(len(docs))])
        for k, name in enumerate(workloads.TRACES):
            assert sha(res[0][k]) == FX[name]["merged_sha256"], name
            assert sha(res[1][k]) == FX[name]["half_sha256"], name
        hb, ho = _arena(res[1])
        sv, svo, st = e.state_vector_host(hb, ho)
        assert not st.any()
        svs = [sv[int(svo[d]):int(svo[d + 1])].tobytes() for d in range(len(res[1]))]
        for k, name in enumerate(workloads.TRACES):
            assert sha(svs[k]) == FX[name]["sv_half_sha256"], name
        fb, fo = _arena(res[0])
        sb, so = _arena(svs)
        df, dfo, st = e.diff_host(fb, fo, sb, so)
        assert not st.any()
        for k, name in enumerate(workloads.TRACES):
            assert sha(df[int(dfo[k]):int(dfo[k + 1])]) == FX[name]["diff_sha256"], name
    finally:
        e.close()
