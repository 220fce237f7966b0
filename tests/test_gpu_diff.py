"""GPU parity for diff_updates_v1 and encode_state_vector_from_update_v1
(yrs/src/alt.rs:54-81): the HIP plan/execute kernels through the C ABI against the
CPU oracle, byte for byte and status for status — reference KATs, Yjs fixtures,
C5-style compacted documents with drawn remote state vectors, documents that take
the length-sized re-plan pass (many clients / DeleteSet entries / unsquashed ranges),
and corrupted inputs."""
import json
import os

import numpy as np
import pytest

import workloads
from conftest import ROOT
from test_oracle_kats import ALT_DIFF, ALT_MERGE_1, ALT_MERGE_2, ALT_SV, COMPAT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["ring", "lane", "wave"])
def engine(request):
    """Every test runs under each common-shape planner (env YMERGE_PLANNER, read at engine
    creation): k_plan_ring, k_plan_lane (+ k_plan_wave for long updates), k_plan_wave for every
    document; the shapes each one hands over go to the general k_plan either way."""
    import ymerge
    old = os.environ.get("YMERGE_PLANNER")
    os.environ["YMERGE_PLANNER"] = request.param
    try:
        e = ymerge.Engine(0)
    finally:
        if old is None:
            del os.environ["YMERGE_PLANNER"]
        else:
            os.environ["YMERGE_PLANNER"] = old
    yield e
    e.close()


def arena(items):
    parts = [np.frombuffer(bytes(x), np.uint8) for x in items]
    lens = [len(p) for p in parts]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = np.concatenate(parts) if parts and sum(lens) else np.zeros(0, np.uint8)
    return data, off


def compare(name, out, off, st, exp, eoff, est):
    bad = np.nonzero(st != est)[0]
    assert len(bad) == 0, f"{name}: status mismatch at {bad[:10]}: gpu {st[bad[:10]]} oracle {est[bad[:10]]}"
    for d in range(len(st)):
        g = out[int(off[d]):int(off[d + 1])].tobytes()
        e = exp[int(eoff[d]):int(eoff[d + 1])]
        if g != e:
            k = next((i for i in range(min(len(g), len(e))) if g[i] != e[i]), min(len(g), len(e)))
            pytest.fail(f"{name} doc {d}: first diff at {k} (gpu {len(g)} B, oracle {len(e)} B)\n"
                        f"gpu    {g[max(0, k - 16):k + 16].hex()}\noracle {e[max(0, k - 16):k + 16].hex()}")


def check_sv(engine, oracle, updates):
    data, off = arena(updates)
    out, o, st = engine.state_vector_host(data, off)
    exp, eoff, est = oracle.sv_batch(data, off, threads=8)
    compare("sv", out, o, st, exp, eoff, est)


def check_diff(engine, oracle, updates, svs):
    data, off = arena(updates)
    sv, soff = arena(svs)
    out, o, st = engine.diff_host(data, off, sv, soff)
    exp, eoff, est = oracle.diff_batch(data, off, sv, soff, threads=8)
    compare("diff", out, o, st, exp, eoff, est)
    return st


def test_alt_kats_single_doc_abi():
    import ymerge
    u, exp = ALT_SV
    assert list(ymerge.encode_state_vector_from_update_v1(bytes(u))) == exp
    u, sv, exp = ALT_DIFF
    assert list(ymerge.diff_updates_v1(bytes(u), bytes(sv))) == exp
    for u in COMPAT.values():
        assert ymerge.diff_updates_v1(bytes(u), b"\x00") == bytes(u)
    with pytest.raises(ymerge.YrsError) as ei:
        ymerge.diff_updates_v1(b"", b"\x00")
    assert ei.value.code == 3
    with pytest.raises(ymerge.YrsError) as ei:
        ymerge.encode_state_vector_from_update_v1(bytes([0x80] * 12))
    assert ei.value.code == 2


def _fixtures():
    with open(os.path.join(ROOT, "tests", "golden", "yjs_fixtures.json")) as f:
        return json.load(f)["cases"]


def test_yjs_fixtures(engine, oracle):
    ups, docs, svs = [], [], []
    for c in _fixtures():
        u = [bytes.fromhex(h) for h in c["updates"]]
        ups += u
        docs.append(bytes.fromhex(c["yjs_merge"]))
        for dd in c["diffs"]:
            docs.append(bytes.fromhex(c["yjs_merge"]))
            svs.append(bytes.fromhex(dd["sv"]))
    check_sv(engine, oracle, ups + docs)
    # every fixture update and merge against every fixture state vector it carries, plus {}
    pairs_u = docs[: len(_fixtures())] + docs[len(_fixtures()):] + ups
    pairs_s = [b"\x00"] * len(_fixtures()) + svs + [b"\x00"] * len(ups)
    check_diff(engine, oracle, pairs_u, pairs_s)


def test_kat_edge_cases(engine, oracle):
    u = [bytes(x) for x in (ALT_MERGE_1[0], ALT_MERGE_1[2], ALT_MERGE_2[2], ALT_DIFF[0], ALT_SV[0])]
    u += [bytes(v) for v in COMPAT.values()]
    edge = [b"", b"\x00", b"\x00\x00", bytes([0x80] * 12), bytes([1, 1, 5, 0, 0x0C, 1, 0]), bytes([0, 0, 7]),
            bytes([1, 0, 5, 3, 0]), bytes([2, 1, 5, 0, 0, 3, 1, 5, 3, 10, 2, 0]),  # client repeated, GC, Skip
            bytes([1, 2, 7, 0, 0, 2, 10, 3, 0])]
    check_sv(engine, oracle, u + edge)
    svs = [b"\x00", bytes([1, 5, 1]), bytes([1, 5, 3]), bytes([2, 5, 1, 5, 9]), b"", bytes([0x80] * 3),
           bytes([1, 0xDC, 0xF0, 0xED, 0xAC, 0x0F, 2]), bytes([5, 1, 1])]
    us, ss = [], []
    for a in u + edge:
        for s in svs:
            us.append(a)
            ss.append(s)
    check_diff(engine, oracle, us, ss)


def _c5(oracle, n_docs, ops, seed, **kw):
    b = workloads.text_docs(n_docs, ops, seed=seed, **kw)
    m, moff, mst = oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=8)
    return workloads.compacted_docs(m, moff, mst, seed=seed,
                                    sv_fn=lambda d, o: oracle.sv_batch(d, o, threads=8))


def test_c5_compacted_docs(engine, oracle):
    c5 = _c5(oracle, 1500, 1000, 0x5713)
    out, o, st = engine.diff_host(c5.data, c5.upd_off, c5.sv, c5.sv_off)
    exp, eoff, est = oracle.diff_batch(c5.data, c5.upd_off, c5.sv, c5.sv_off, threads=8)
    compare("c5", out, o, st, exp, eoff, est)
    assert (st == 0).all()
    s = engine.stats()
    assert s["docs_exact"] == 0  # no document needed the length-sized re-plan
    out, o, st = engine.state_vector_host(c5.data, c5.upd_off)
    exp, eoff, est = oracle.sv_batch(c5.data, c5.upd_off, threads=8)
    compare("c5-sv", out, o, st, exp, eoff, est)


def test_c5_many_clients_replan(engine, oracle):
    """> 8 clients per document: every document takes the length-sized re-plan pass."""
    c5 = _c5(oracle, 200, 400, 99, min_clients=9, max_clients=14)
    out, o, st = engine.diff_host(c5.data, c5.upd_off, c5.sv, c5.sv_off)
    exp, eoff, est = oracle.diff_batch(c5.data, c5.upd_off, c5.sv, c5.sv_off, threads=8)
    compare("c5-many", out, o, st, exp, eoff, est)
    assert engine.stats()["docs_exact"] == 200
    check_sv(engine, oracle, [c5.update(d) for d in range(c5.n_docs)])


def test_raw_updates_and_delete_heavy(engine, oracle):
    """Per-op updates of C2 and the C4 inputs (GC'd snapshots, Skips) as single updates."""
    b = workloads.text_docs(20, 200, seed=3)
    c4 = workloads.delete_heavy_docs(6, ops_per_doc=800, seed=4)
    ups = [b.data[int(b.upd_off[u]):int(b.upd_off[u + 1])].tobytes() for u in range(0, b.n_updates, 7)]
    ups += [c4.data[int(c4.upd_off[u]):int(c4.upd_off[u + 1])].tobytes() for u in range(c4.n_updates)]
    check_sv(engine, oracle, ups)
    m, moff, _ = oracle.merge_batch(c4.data, c4.upd_off, c4.doc_upd, mode=1, threads=8)
    merged = [m[int(moff[d]):int(moff[d + 1])] for d in range(c4.n_docs)]
    svs = [oracle.encode_state_vector_from_update_v1(x) for x in merged]
    rng = np.random.default_rng(5)
    us, ss = [], []
    for x, s in zip(merged + ups[:300], svs + [b"\x00"] * 300):
        pairs = workloads.parse_sv(s)
        for _ in range(3):
            us.append(x)
            ss.append(workloads.encode_sv([(c, int(rng.integers(0, k + 2))) for c, k in pairs]))
    check_diff(engine, oracle, us, ss)


def _ds_update(entries, blocks=b"\x00"):
    b = bytearray(blocks) + workloads._var(len(entries))
    for c, rs in entries:
        b += workloads._var(c) + workloads._var(len(rs))
        for s, n in rs:
            b += workloads._var(s) + workloads._var(n)
    return bytes(b)


def test_deleteset_tables(engine, oracle):
    """DeleteSet re-encode: table order with many entries (re-plan), repeated clients
    (HashMap::insert replacement), unsquashed / overlapping / adjacent / empty ranges."""
    rng = np.random.default_rng(8)
    ups = []
    for n_ent in (0, 1, 2, 5, 8, 9, 17, 40, 100):
        for rep in range(4):
            ents = []
            for _ in range(n_ent):
                c = int(rng.integers(0, 6)) if rep == 1 else int(rng.integers(0, 2 ** 32))
                k = int(rng.integers(0, 5))
                rs = [(int(rng.integers(0, 60)), int(rng.integers(0, 9))) for _ in range(k)]
                if rep == 2:
                    rs.sort()
                ents.append((c, rs))
            ups.append(_ds_update(ents))
            ups.append(_ds_update(ents, bytes(ALT_MERGE_1[2])[:-1]))
    check_sv(engine, oracle, ups)
    check_diff(engine, oracle, ups, [b"\x00"] * len(ups))


def test_fuzz_corruptions(engine, oracle):
    rng = np.random.default_rng(4321)
    base = [bytes.fromhex(c["yjs_merge"]) for c in _fixtures()] + [bytes(v) for v in COMPAT.values()]
    us, ss = [], []
    for u in base:
        for _ in range(8):
            m = bytearray(u)
            for _ in range(rng.integers(1, 4)):
                if not m:
                    break
                i = int(rng.integers(len(m)))
                op = rng.integers(3)
                if op == 0:
                    m[i] = int(rng.integers(256))
                elif op == 1:
                    del m[i:]
                else:
                    m.insert(i, int(rng.integers(256)))
            us.append(bytes(m))
            sv = bytearray(oracle.encode_state_vector_from_update_v1(u)) if rng.random() < 0.8 else bytearray(b"\x00")
            if sv and rng.random() < 0.3:
                sv[int(rng.integers(len(sv)))] = int(rng.integers(256))
            ss.append(bytes(sv))
    check_sv(engine, oracle, us)
    check_diff(engine, oracle, us, ss)
