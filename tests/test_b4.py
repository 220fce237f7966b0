"""The reference's giant single update, assets/bench-input/b4-update.bin (400,972 B, one
client, 12,387 blocks with the rest of a LaTeX paper's editing history; used by
yrs/benches/benches.rs:456-473), through merge_updates_v1 / encode_state_vector_from_update_v1
/ diff_updates_v1 (yrs/src/alt.rs:15-81).  The reference holds no expected outputs for it, so
the CPU test pins the oracle's reading of it (status 0, one client, the state vector's clock
= the sum of the decoded block lengths) and the GPU tests compare the HIP path with the
oracle byte for byte, including remote state vectors that cut blocks (spliced first block)."""
import numpy as np
import pytest

import corpus
from test_gpu_parity import batch_of, check_batch


def _var(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        out.append(b | (0x80 if x else 0))
        if not x:
            return bytes(out)


def sv_bytes(pairs):
    """StateVector::encode layout (state_vector.rs:126-134): count, then (client, clock) varints."""
    return _var(len(pairs)) + b"".join(_var(c) + _var(k) for c, k in pairs)


def _remote_svs(client, clock):
    cuts = [0, 1, 2, 7, clock // 3, clock // 2 + 1, clock - 5, clock - 1, clock, clock + 10]
    svs = [b"\x00"] + [sv_bytes([(client, c)]) for c in cuts] + [sv_bytes([(client + 1, 5), (client, clock // 4)])]
    return svs


def test_b4_oracle_reading(oracle):
    u = corpus.b4_update()
    assert len(u) == 400_972
    st, m = oracle.status_of(oracle.merge_updates_v1, [u])
    assert st == 0 and len(m) > 0
    sv = oracle.parse_sv(oracle.encode_state_vector_from_update_v1(u))
    assert len(sv) == 1
    (client, clock), = sv
    # diff against the document's own state vector: no blocks, only the DeleteSet
    d = oracle.diff_updates_v1(u, oracle.encode_state_vector_from_update_v1(u))
    assert d[0] == 0 and oracle.ds_offset(d) == 1
    # merging the update with itself changes nothing (duplicates are covered blocks)
    assert oracle.merge_updates_v1([u, u]) == m
    # the oracle's merge is a fixed point
    assert oracle.merge_updates_v1([m]) == oracle.merge_updates_v1([oracle.merge_updates_v1([m])])
    assert clock == 182_315 and client == 992_525_821


@pytest.mark.gpu
def test_b4_merge_gpu(oracle):
    import ymerge
    u = corpus.b4_update()
    eng = ymerge.Engine(0)
    try:
        check_batch(eng, oracle, batch_of([[u], [u, u], [u[:200_000]], [u, b"\x00\x00"]]))
        st = eng.stats()
        assert st["docs_exact"] == 0, st
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("planner", ["grid", "ring", "lane", "wave"])
def test_b4_sv_and_diff_gpu(oracle, planner):
    """b4 and its merge through the long-update grid path (ylong.hip: the parallel parse, then a
    lane per block) and, with it turned off, through each planner (the merged form is canonical,
    375 KB: under "lane" it is a k_plan_wave document; b4 itself has 7-byte client varints, which
    the common-shape planners hand to k_plan)."""
    from test_gpu_diff import check_diff, check_sv
    from test_gpu_parity import engine_with
    u = corpus.b4_update()
    m = oracle.merge_updates_v1([u])
    (client, clock), = oracle.parse_sv(oracle.encode_state_vector_from_update_v1(u))
    env = {} if planner == "grid" else {"YMERGE_PLANNER": planner, "YMERGE_LONG_GRID": 0}
    eng = engine_with(**env)
    try:
        check_sv(eng, oracle, [u, m])
        svs = _remote_svs(client, clock)
        check_diff(eng, oracle, [u] * len(svs) + [m] * len(svs), svs + svs)
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [1, 0])
def test_b4_merge_paths(oracle, grid):
    """merge_updates_v1([b4]) on the long-update grid path and, turned off, on the tiled kernel;
    also with the parallel parse off (every long update walked by k_decode_huge)."""
    import ymerge
    from test_gpu_parity import engine_with
    u = corpus.b4_update()
    for env in ({"YMERGE_LONG_GRID": grid}, {"YMERGE_LONG_PARSE": grid}):
        eng = engine_with(**env)
        try:
            check_batch(eng, oracle, batch_of([[u], [u[:5000]], [u], [u, b"\x00\x00"]]))
            st = eng.stats()
            if grid:
                assert st["docs_giant"] >= 2, st  # the two [u] documents on the grid path
        finally:
            eng.close()
