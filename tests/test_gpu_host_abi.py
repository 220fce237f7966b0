"""The server-facing host-memory batch entries of the C ABI (include/ymerge.h, "batched,
host memory": host pointers in, a library-owned ymerge_batch_result out), each against
the CPU oracle byte for byte; and the C++ FFI test binary (tests/ffi), which links
libymerge.so the way the reference's tests-ffi/main.cpp:38-50 links yffi."""
import os
import subprocess

import numpy as np
import pytest

import workloads
from conftest import ROOT
from test_gpu_parity import batch_of
from test_oracle_kats import ALT_DIFF, ALT_MERGE_1, ALT_MERGE_2, ALT_SV, COMPAT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    import ymerge
    e = ymerge.Engine(0)
    yield e
    e.close()


def _same(got, exp):
    out, off, st = got
    eb, eoff, est = exp
    assert np.array_equal(st, est), (np.nonzero(st != est)[0][:8], st[st != est][:8], est[st != est][:8])
    assert np.array_equal(off.astype(np.uint64), np.asarray(eoff, np.uint64))
    assert out.tobytes() == bytes(eb)


def _docs():
    docs = [[bytes(ALT_MERGE_1[0]), bytes(ALT_MERGE_1[1])], [bytes(ALT_MERGE_2[0]), bytes(ALT_MERGE_2[1])],
            [], [b""], [bytes([0x80] * 12)]] + [[bytes(u)] for u in COMPAT.values()]
    b = workloads.text_docs(200, 150, seed=11)
    docs += [b.doc_updates(d) for d in range(b.n_docs)]
    return docs


def test_merge_v1_batch(engine, oracle):
    b = batch_of(_docs())
    got = engine.host_batch("ymerge_updates_v1_batch", b.data, b.upd_off, len(b.upd_off) - 1, b.doc_upd)
    _same(got, oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=8))


def test_merge_v2_batch(engine, oracle):
    docs = [ups for ups in _docs() if all(oracle.status_of(oracle.convert_update_v1_to_v2, u)[0] == 0 for u in ups)]
    docs = [[oracle.convert_update_v1_to_v2(u) for u in ups] for ups in docs]
    b = batch_of(docs)
    got = engine.host_batch("ymerge_updates_v2_batch", b.data, b.upd_off, len(b.upd_off) - 1, b.doc_upd)
    _same(got, oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=8, version=2))


def _merged(oracle):
    b = batch_of(_docs())
    m, moff, mst = oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=8)
    keep = [d for d in range(b.n_docs) if mst[d] == 0]
    ups = [m[int(moff[d]):int(moff[d + 1])] for d in keep]
    ups += [bytes(ALT_DIFF[0]), bytes(ALT_SV[0]), b"", bytes([1, 1])]  # + KAT inputs and malformed ones
    off = np.cumsum([0] + [len(u) for u in ups]).astype(np.uint64)
    return np.frombuffer(b"".join(ups), np.uint8), off


def _remote(oracle, ub, uoff):
    sv, svoff, st = oracle.sv_batch(ub, uoff, threads=8)
    svs = [bytes(sv[int(svoff[d]):int(svoff[d + 1])]) if st[d] == 0 else b"\x00" for d in range(len(uoff) - 1)]
    sva = np.frombuffer(b"".join(svs), np.uint8)
    rsv, rsv_off = workloads.remote_svs(sva, np.cumsum([0] + [len(x) for x in svs]).astype(np.uint64))
    svs = [rsv[int(rsv_off[d]):int(rsv_off[d + 1])].tobytes() for d in range(len(uoff) - 1)]
    svs[-4] = bytes(ALT_DIFF[1])
    svs[-1] = b"\x05"  # truncated state vector
    return np.frombuffer(b"".join(svs), np.uint8), np.cumsum([0] + [len(s) for s in svs]).astype(np.uint64)


def test_sv_and_diff_v1_batch(engine, oracle):
    ub, uoff = _merged(oracle)
    got = engine.host_batch("yencode_state_vector_from_update_v1_batch", ub, uoff)
    _same(got, oracle.sv_batch(ub, uoff, threads=8))
    sb, soff = _remote(oracle, ub, uoff)
    got = engine.host_batch("ydiff_updates_v1_batch", ub, uoff, sb, soff)
    exp = oracle.diff_batch(ub, uoff, sb, soff, threads=8)
    _same(got, exp)
    d = len(uoff) - 1 - 4  # the ALT_DIFF KAT document (yrs/src/alt.rs:144-160)
    assert list(got[0][int(got[1][d]):int(got[1][d + 1])]) == ALT_DIFF[2]


def test_sv_and_diff_v2_batch(engine, oracle):
    ub, uoff = _merged(oracle)
    ups = [ub[int(uoff[d]):int(uoff[d + 1])].tobytes() for d in range(len(uoff) - 1)]
    ups = [oracle.convert_update_v1_to_v2(u) for u in ups[:-2]]
    u2 = np.frombuffer(b"".join(ups), np.uint8)
    o2 = np.cumsum([0] + [len(u) for u in ups]).astype(np.uint64)
    got = engine.host_batch("yencode_state_vector_from_update_v2_batch", u2, o2)
    _same(got, oracle.sv_batch(u2, o2, threads=8, version=2))
    sv2, sv2off, _ = oracle.sv_batch(u2, o2, threads=8, version=2)
    got = engine.host_batch("ydiff_updates_v2_batch", u2, o2, np.frombuffer(sv2, np.uint8), sv2off)
    _same(got, oracle.diff_batch(u2, o2, np.frombuffer(sv2, np.uint8), sv2off, threads=8, version=2))


def test_sync_batch(engine, oracle):
    ub, uoff = _merged(oracle)
    n = len(uoff) - 1
    got = engine.host_batch("ysync_step1_v1_batch", ub, uoff)
    ups = [ub[int(uoff[d]):int(uoff[d + 1])].tobytes() for d in range(n)]
    exp1 = [oracle.status_of(oracle.sync_step1_v1, u) for u in ups]
    for d in range(n):
        st, data = exp1[d]
        assert got[2][d] == st, d
        assert got[0][int(got[1][d]):int(got[1][d + 1])].tobytes() == (data or b""), d
    msgs = [exp1[d][1] or b"\x00\x00\x01\x00" for d in range(n)]
    msgs[0] = b"\x00\x02\x00"  # a SyncStep2 message from the client: UNSUPPORTED
    mb = np.frombuffer(b"".join(msgs), np.uint8)
    moff = np.cumsum([0] + [len(m) for m in msgs]).astype(np.uint64)
    got = engine.host_batch("ysync_step2_v1_batch", ub, uoff, mb, moff)
    for d in range(n):
        st, data = oracle.status_of(oracle.sync_step2_v1, ups[d], msgs[d])
        assert got[2][d] == st, d
        assert got[0][int(got[1][d]):int(got[1][d + 1])].tobytes() == (data or b""), d


def test_c2_batch_through_host_entry(engine, oracle):
    b = workloads.text_docs(1000, 400, seed=5)
    got = engine.host_batch("ymerge_updates_v1_batch", b.data, b.upd_off, len(b.upd_off) - 1, b.doc_upd)
    _same(got, oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=8))


def test_ffi_binary():
    exe = os.path.join(ROOT, "tests", "ffi", "ymerge_ffi_test")
    assert os.path.exists(exe), "tests/ffi/ymerge_ffi_test not built (__graft_entry__.build())"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout[-2000:])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "0 failed" in r.stdout


@pytest.mark.parametrize("n_ctx", [1, 2, 3])
def test_multi_context_merge_and_diff(oracle, n_ctx):
    """ymerge_updates_v1_batch_multi / ydiff_updates_v1_batch_multi with n_ctx contexts on
    device 0 (the sharding logic is device-count independent): input order, byte-exact."""
    import ymerge
    engines = [ymerge.Engine(0) for _ in range(n_ctx)]
    try:
        b = batch_of(_docs())
        exp = oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=8)
        _same(ymerge.merge_multi(engines, b.data, b.upd_off, b.doc_upd), exp)
        ids = np.arange(1000, 1000 + b.n_docs, dtype=np.uint64)[::-1].copy()
        _same(ymerge.merge_multi(engines, b.data, b.upd_off, b.doc_upd, doc_ids=ids), exp)
        ub, uoff = _merged(oracle)
        sb, soff = _remote(oracle, ub, uoff)
        _same(ymerge.diff_multi(engines, ub, uoff, sb, soff), oracle.diff_batch(ub, uoff, sb, soff, threads=8))
    finally:
        for e in engines:
            e.close()


def test_pipelined_host_entry(engine, oracle):
    """A host batch above 96 MB takes the pipelined path (document groups of ~48 MB: H2D,
    merge and D2H overlapped); GPU == oracle, documents in input order."""
    b = workloads.text_docs(4000, 1000, seed=21)
    assert b.n_bytes >= 96 << 20
    got = engine.host_batch("ymerge_updates_v1_batch", b.data, b.upd_off, len(b.upd_off) - 1, b.doc_upd)
    _same(got, oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=8))
