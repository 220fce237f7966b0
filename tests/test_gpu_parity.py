"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle, byte for
byte, on the reference KATs, the Yjs-generated fixtures, synthetic batches of
every BASELINE config, error/fuzz cases and the full automerge-paper trace."""
import json
import os

import numpy as np
import pytest

import workloads
from conftest import ROOT
from test_oracle_kats import ALT_DIFF, ALT_MERGE_1, ALT_MERGE_2, ALT_SV, COMPAT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    import ymerge
    e = ymerge.Engine(0)
    yield e
    e.close()


def run_batch(engine, batch):
    return engine.merge_host(batch.data, batch.upd_off, batch.doc_upd)


def check_batch(engine, oracle, batch, mode=1):
    out, off, st = run_batch(engine, batch)
    exp, eoff, est = oracle.merge_batch(batch.data, batch.upd_off, batch.doc_upd, mode=mode, threads=8)
    bad = np.nonzero(st != est)[0]
    assert len(bad) == 0, f"status mismatch at docs {bad[:10]}: gpu {st[bad[:10]]} oracle {est[bad[:10]]}"
    for d in range(batch.n_docs):
        g = out[int(off[d]):int(off[d + 1])].tobytes()
        e = exp[int(eoff[d]):int(eoff[d + 1])]
        if g != e:
            k = next((i for i in range(min(len(g), len(e))) if g[i] != e[i]), min(len(g), len(e)))
            pytest.fail(f"doc {d}: first byte diff at {k} (gpu len {len(g)}, oracle len {len(e)})\n"
                        f"gpu    {g[max(0, k - 16):k + 16].hex()}\noracle {e[max(0, k - 16):k + 16].hex()}")
    return out, off, st


def batch_of(docs):
    parts, offs, dus, tot = [], [0], [0], 0
    for ups in docs:
        for u in ups:
            parts.append(np.frombuffer(bytes(u) or b"", dtype=np.uint8))
            tot += len(u)
            offs.append(tot)
        dus.append(len(offs) - 1)
    data = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return workloads.Batch(data, np.array(offs, np.uint64), np.array(dus, np.uint64))


def test_alt_kats_single_doc_abi():
    import ymerge
    for a, b, exp in (ALT_MERGE_1, ALT_MERGE_2):
        assert list(ymerge.merge_updates_v1([bytes(a), bytes(b)])) == exp
    for u in COMPAT.values():
        assert ymerge.merge_updates_v1([bytes(u)]) == bytes(u)
    with pytest.raises(ymerge.YrsError) as ei:
        ymerge.merge_updates_v1([b""])
    assert ei.value.code == 3


def test_yjs_fixture_batch(engine, oracle):
    with open(os.path.join(ROOT, "tests", "golden", "yjs_fixtures.json")) as f:
        cases = json.load(f)["cases"]
    docs = [[bytes.fromhex(h) for h in c["updates"]] for c in cases]
    check_batch(engine, oracle, batch_of(docs))


def test_edge_docs(engine, oracle):
    docs = [[], [b""], [bytes([0, 0])], [bytes([0x80] * 12)], [bytes([1, 1, 5, 0, 0x0C, 1, 0])],
            [bytes(ALT_MERGE_1[0]), b"\x01"], [bytes(ALT_MERGE_1[0])] * 5,
            [bytes(ALT_MERGE_2[0]), bytes(ALT_MERGE_2[1])], [bytes(ALT_MERGE_2[1]), bytes(ALT_MERGE_2[0])]]
    check_batch(engine, oracle, batch_of(docs))


def test_fuzz_corruptions(engine, oracle):
    with open(os.path.join(ROOT, "tests", "golden", "yjs_fixtures.json")) as f:
        cases = json.load(f)["cases"]
    rng = np.random.default_rng(1234)
    docs = []
    for c in cases:
        ups = [bytearray.fromhex(h) for h in c["updates"]][:40]
        for _ in range(6):
            mut = [bytearray(u) for u in ups]
            for _ in range(rng.integers(1, 4)):
                u = mut[rng.integers(len(mut))]
                if len(u) == 0:
                    continue
                op = rng.integers(3)
                i = rng.integers(len(u))
                if op == 0:
                    u[i] = rng.integers(256)
                elif op == 1:
                    del u[i:]
                else:
                    u.insert(i, rng.integers(256))
            docs.append([bytes(u) for u in mut])
    check_batch(engine, oracle, batch_of(docs))


def test_c2_batch(engine, oracle):
    check_batch(engine, oracle, workloads.text_docs(300, 1000))


def test_c2_many_clients(engine, oracle):
    check_batch(engine, oracle, workloads.text_docs(200, 400, seed=77, min_clients=5, max_clients=12))


def test_c3_zipf_batch(engine, oracle):
    check_batch(engine, oracle, workloads.zipf_docs(2000, seed=0x5EED))


def test_c4_delete_heavy(engine, oracle):
    check_batch(engine, oracle, workloads.delete_heavy_docs(24, ops_per_doc=2000), mode=1)


def test_exact_engine_only(oracle):
    """Same C2/C4 inputs through the exact per-document engine alone (fast path off)."""
    import ymerge
    os.environ["YMERGE_FAST_THREADS"] = "0"
    try:
        e = ymerge.Engine(0)
    finally:
        del os.environ["YMERGE_FAST_THREADS"]
    try:
        check_batch(e, oracle, workloads.text_docs(100, 500, seed=5))
        check_batch(e, oracle, workloads.delete_heavy_docs(6, ops_per_doc=1500, seed=9))
    finally:
        e.close()


def engine_with(**env):
    """An Engine created under the given YMERGE_* environment knobs (read at creation)."""
    import ymerge
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return ymerge.Engine(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("threads", ["256", "512", "1024"])
def test_fast_path_workgroup_sizes(oracle, threads):
    """k_decode + k_fast_merge alone (k_lean off) at every workgroup size."""
    e = engine_with(YMERGE_FAST_THREADS=threads, YMERGE_LEAN=0)
    try:
        check_batch(e, oracle, workloads.text_docs(150, 1000, seed=11))
    finally:
        e.close()


def test_fast_path_coverage(engine, oracle):
    """C2 documents must all be written by k_lean (no silent hand-over to the slower paths)."""
    check_batch(engine, oracle, workloads.text_docs(500, 1000, seed=21))
    st = engine.stats()
    assert st["docs_exact"] == 0 and st["docs_lean"] == 500 and st["docs_fast"] == 0


def test_fast_path_coverage_without_lean(oracle):
    """With k_lean off, C2 documents stay on k_fast_merge (no exact-engine fallback)."""
    e = engine_with(YMERGE_LEAN=0)
    try:
        check_batch(e, oracle, workloads.text_docs(300, 1000, seed=21))
        st = e.stats()
        assert st["docs_exact"] == 0 and st["docs_fast"] == 300 and st["docs_lean"] == 0
    finally:
        e.close()


def test_c1_automerge_trace(engine, oracle):
    b, _ = workloads.trace_updates()
    check_batch(engine, oracle, b, mode=1)


def _var(x):
    out = bytearray()
    while True:
        b, x = x & 0x7F, x >> 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _ds_update(entries):
    """A v1 update with no blocks and the given DeleteSet [(client, [(start, len)])]."""
    b = bytearray(_var(0)) + _var(len(entries))
    for c, rs in entries:
        b += _var(c) + _var(len(rs))
        for s, n in rs:
            b += _var(s) + _var(n)
    return bytes(b)


def ds_heavy_docs(seed):
    """Documents whose updates carry many DeleteSet entries (around the 14-entry
    in-register table, the 8 entries whose table codes k_decode packs into the record,
    and the former 64-entry limit), with repeated clients inside
    one update (HashMap::insert replacement, id_set.rs decode)."""
    rng = np.random.default_rng(seed)
    docs = []
    for n_ent in (2, 3, 7, 8, 9, 13, 14, 15, 40, 56, 57, 64, 65, 120, 300):  # 8: packed table codes
        for rep in range(3):
            ups = []
            for _ in range(4):
                ents = []
                for _ in range(n_ent):
                    if rng.random() < 0.3:
                        c = int(rng.integers(0, max(4, n_ent // 2)))
                    else:
                        c = int(rng.integers(0, 2 ** 32))
                    rs = [(int(rng.integers(0, 1000)), int(rng.integers(1, 20))) for _ in range(rng.integers(1, 3))]
                    ents.append((c, rs))
                ups.append(_ds_update(ents))
            if rep:
                ups.append(bytes(ALT_MERGE_1[rep - 1]))
            docs.append(ups)
    return docs


def test_ds_heavy_updates(engine, oracle):
    check_batch(engine, oracle, batch_of(ds_heavy_docs(31)))


def test_ds_heavy_updates_exact_engine(oracle):
    import ymerge
    os.environ["YMERGE_FAST_THREADS"] = "0"
    try:
        e = ymerge.Engine(0)
    finally:
        del os.environ["YMERGE_FAST_THREADS"]
    try:
        check_batch(e, oracle, batch_of(ds_heavy_docs(32)))
    finally:
        e.close()


def _root_text_update(client, clock, s):
    """One v1 update: a single String item with no origins under root type "t"
    (yrs/src/update.rs:433-488 decode_block; parent info 1 = root name)."""
    body = bytes([0x04]) + _var(1) + _var(1) + b"t" + _var(len(s)) + s.encode()
    return _var(1) + _var(1) + _var(client) + _var(clock) + body + _var(0)


def test_large_block_sections(engine, oracle):
    """Block sections around and above the fast path's 20 KB LDS stage (staged and
    direct-to-HBM writers), updates in shuffled order from two clients."""
    rng = np.random.default_rng(0x57A6E)
    docs = []
    for n in (150, 300, 330, 360, 480):
        ups = []
        for c in (3, 9):
            clock = 0
            for i in range(n // 2):
                s = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, 60))
                ups.append(_root_text_update(c, clock, s))
                clock += len(s)
        order = rng.permutation(len(ups))
        docs.append([ups[i] for i in order])
    check_batch(engine, oracle, batch_of(docs))
    st = engine.stats()
    assert st["docs_exact"] == 0


def test_deleteset_union_shapes(engine, oracle):
    """DeleteSet unions through both fast-path variants: the bitmap (non-empty ranges in
    windows up to 32768 clocks) and the range sort (empty ranges [c, c), wide windows),
    with touching / overlapping / nested / duplicate ranges and several clients."""
    rng = np.random.default_rng(77)
    docs = []
    for case in range(60):
        ups = []
        span = [40, 300, 5000, 40000, 1 << 31][case % 5]
        for _ in range(int(rng.integers(2, 60))):
            ents = []
            for c in rng.choice([3, 9, 27, 81, 1 << 30], size=int(rng.integers(1, 4)), replace=False):
                rs = []
                for _ in range(int(rng.integers(1, 4))):
                    s = int(rng.integers(0, span))
                    n = int(rng.integers(0 if case % 7 == 0 else 1, 40))
                    rs.append((s, n))
                ents.append((int(c), rs))
            ups.append(_ds_update(ents))
        ups.append(_root_text_update(5, 0, "x" * int(rng.integers(1, 30))))
        docs.append([ups[i] for i in rng.permutation(len(ups))])
    check_batch(engine, oracle, batch_of(docs))
