"""GPU parity of the lib0 v2 path (yv2.hip: DecoderV2 -> engine -> EncoderV2) against the
oracle's v2 restatement (oracle/yrs_oracle_v2.c, pinned in tests/test_v2.py): the
compatibility_tests.rs v2 payloads, the Yjs v2 fixtures (text, UTF-16, maps, arrays,
rich text with Format/Embed, xml, two clients), v2 forms of C2 / overlapping documents
(fast path, tiled kernel overlap mode), the reference corpus, and corrupted updates
(status for status)."""
import json
import os

import numpy as np
import pytest

import workloads
from conftest import ROOT
from overlaps import overlap_docs
from test_gpu_parity import batch_of

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden")
V2_HEADER = bytes([0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0])


@pytest.fixture(scope="module")
def engine():
    import ymerge
    e = ymerge.Engine(0)
    yield e
    e.close()


def _check_merge(engine, oracle, docs):
    b = batch_of(docs)
    out, off, st = engine.merge_host(b.data, b.upd_off, b.doc_upd, version=2)
    exp, eoff, est = oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=8, version=2)
    bad = np.nonzero(st != est)[0]
    assert len(bad) == 0, f"status mismatch at {bad[:10]}: gpu {st[bad[:10]]} oracle {est[bad[:10]]}"
    for d in range(len(docs)):
        g = out[int(off[d]):int(off[d + 1])].tobytes()
        e = exp[int(eoff[d]):int(eoff[d + 1])]
        assert g == e, f"doc {d}: gpu {g[:48].hex()} oracle {e[:48].hex()}"
    return [out[int(off[d]):int(off[d + 1])].tobytes() for d in range(len(docs))], st


def _arena(bufs):
    off = np.zeros(len(bufs) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in bufs])
    return np.frombuffer(b"".join(bufs) or b"\0", np.uint8)[: int(off[-1])], off


def _check_sv_diff(engine, oracle, updates, svs):
    ub, uo = _arena(updates)
    sv, svo, st = engine.state_vector_host(ub, uo, version=2)
    for d, u in enumerate(updates):
        code, exp = oracle.status_of(oracle.encode_state_vector_from_update_v2, u)
        assert st[d] == code, (d, st[d], code)
        if not code:
            assert sv[int(svo[d]):int(svo[d + 1])].tobytes() == exp, d
    sb, so = _arena(svs)
    df, dfo, st = engine.diff_host(ub, uo, sb, so, version=2)
    for d, (u, s) in enumerate(zip(updates, svs)):
        code, exp = oracle.status_of(oracle.diff_updates_v2, u, s)
        assert st[d] == code, (d, st[d], code)
        if not code:
            assert df[int(dfo[d]):int(dfo[d + 1])].tobytes() == exp, d


def test_compat_payloads_single_doc_abi(oracle):
    import ymerge
    fx = json.load(open(os.path.join(GOLD, "compat_v2.json")))
    for name, (p1, p2) in fx["pairs"].items():
        p2 = bytes.fromhex(p2)
        assert ymerge.merge_updates_v2([p2]) == p2, name
        assert ymerge.merge_updates_v2([p2, p2]) == p2, name
        assert ymerge.encode_state_vector_from_update_v2(p2) == oracle.encode_state_vector_from_update_v2(p2)
        assert ymerge.diff_updates_v2(p2, V2_HEADER + b"\x00") == p2
    u = bytes.fromhex(fx["utf32_lib0_v2_decoding"])
    assert ymerge.merge_updates_v2([u]) == oracle.merge_updates_v2([u])
    with pytest.raises(ymerge.YrsError) as e:
        ymerge.merge_updates_v2([b""])
    assert e.value.code == 2


def test_yjs_v2_fixtures(engine, oracle):
    cases = json.load(open(os.path.join(GOLD, "yjs_fixtures_v2.json")))["cases"]
    merged, _ = _check_merge(engine, oracle, [[bytes.fromhex(h) for h in c["v2"]] for c in cases])
    svs = [V2_HEADER + bytes.fromhex(c["diffs"][0]["sv"]) for c in cases]
    _check_sv_diff(engine, oracle, merged, svs)


def _v2_docs(oracle, docs):
    out = []
    for ups in docs:
        conv = [oracle.status_of(oracle.convert_update_v1_to_v2, u) for u in ups]
        if all(c == 0 for c, _ in conv):
            out.append([x for _, x in conv])
    return out


def test_c2_docs_v2(engine, oracle):
    b = workloads.text_docs(300, ops_per_doc=400)
    docs = _v2_docs(oracle, [b.doc_updates(d) for d in range(b.n_docs)])
    assert len(docs) == 300
    merged, st = _check_merge(engine, oracle, docs)
    assert not st.any()
    halves = [oracle.merge_updates_v2(d[: len(d) // 2]) for d in docs[:100]]
    svs = [oracle.encode_state_vector_from_update_v2(h) for h in halves]
    _check_sv_diff(engine, oracle, merged[:100], svs)


@pytest.mark.parametrize("seed", [4, 5])
def test_overlap_docs_v2(engine, oracle, seed):
    docs = _v2_docs(oracle, overlap_docs(seed))
    _check_merge(engine, oracle, docs)
    st = engine.stats()
    assert st["docs_overlap"] > 0, st


def test_corpus_v2(engine, oracle):
    import corpus
    docs = _v2_docs(oracle, [ups for ups, *_ in corpus.small_dataset()[::3]])
    assert len(docs) > 1000
    _check_merge(engine, oracle, docs)


def test_corrupted_v2_updates(engine, oracle):
    cases = json.load(open(os.path.join(GOLD, "yjs_fixtures_v2.json")))["cases"]
    rng = np.random.default_rng(99)
    docs = []
    for c in cases:
        ups = [bytearray.fromhex(h) for h in c["v2"]][:30]
        for _ in range(8):
            mut = [bytearray(u) for u in ups]
            for _ in range(rng.integers(1, 4)):
                u = mut[rng.integers(len(mut))]
                if not u:
                    continue
                i = int(rng.integers(len(u)))
                op = rng.integers(3)
                if op == 0:
                    u[i] = int(rng.integers(256))
                elif op == 1:
                    del u[i:]
                else:
                    u.insert(i, int(rng.integers(256)))
            docs.append([bytes(u) for u in mut])
    # column lengths at the usize edge: 2^64 - 1 (start + len overflows: panic), 2^63 - 1 (EOS)
    docs.append([bytes([0] + [0xFF] * 9 + [0x01])])
    docs.append([bytes([0] + [0xFF] * 8 + [0x7F])])
    _check_merge(engine, oracle, docs)
