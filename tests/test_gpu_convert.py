"""yconvert_updates_v1_to_v2_batch_device: every update u becomes merge_updates_v1([u])
re-encoded by EncoderV2 (include/ymerge.h; yrs/src/alt.rs:15-28, Update::encode_v2
yrs/src/updates/encoder.rs:182-528), i.e. Update::merge_updates([decode_v1(u)]).encode_v2().
Checked against the oracle's restatement of exactly that (oracle.merge_updates_v2(...,
inputs_v1=True)).  It is not always Update::decode_v1(u).encode_v2(): merge rewrites
overlapping same-client blocks and adjacent Skips, and a DeleteSet of >= 2 clients comes out
in the merged map's order, not the decoded map's (hashbrown iteration depends on the table's
capacity and insertion order)."""
import pytest

from overlaps import _item, _var, update



def _skip(n):
    return bytes([10]) + _var(n)


def _section(client, clock, blocks):
    return _var(len(blocks)) + _var(client) + _var(clock) + b"".join(blocks)


def _raw_update(sections, ds=b"\x00"):
    return _var(len(sections)) + b"".join(sections) + ds


def edge_updates():
    return [
        # one client in two sections of one update, the second overlapping the first
        # (decode appends both to one block queue; merge slices the covered part,
        # update.rs:611-679)
        update([(5, 0, [("i", "abc")]), (5, 1, [("i", "xyzw")])]),
        update([(7, 2, [("i", "hello")]), (7, 0, [("i", "he")]), (9, 0, [("g", 3)])], [(7, [(0, 2)])]),
        # adjacent Skips inside one section (joined by BlockCarrier::try_squash, update.rs:854)
        _raw_update([_section(3, 0, [_item("ab"), _skip(3), _skip(2), _item("cd")])]),
        _raw_update([_section(3, 4, [_skip(1), _skip(1), _skip(1)]), _section(2, 0, [_item("q")])]),
        # a trailing Skip and an empty section
        _raw_update([_section(11, 0, [_item("z"), _skip(4)]), _section(12, 0, [])]),
    ]


@pytest.mark.gpu
def test_convert_v1_to_v2_device(oracle):
    """Per-op text updates (multi-client DeleteSets included)."""
    import ymerge
    import workloads
    b = workloads.text_docs(20, 100, seed=77, max_clients=3)
    e = ymerge.Engine(0)
    try:
        out, off, st = e.convert_v1_to_v2_host(b.data, b.upd_off)
    finally:
        e.close()
    assert not st.any()
    same = 0
    for i in range(b.n_updates):
        u = bytes(b.data[int(b.upd_off[i]):int(b.upd_off[i + 1])])
        want = oracle.merge_updates_v2([u], inputs_v1=True)
        assert out[int(off[i]):int(off[i + 1])].tobytes() == want, i
        same += want == oracle.convert_update_v1_to_v2(u)
    assert same > 0.9 * b.n_updates  # mostly decode-then-encode too (not the multi-client DeleteSets)


def test_convert_edge_cases_differ_from_decode_encode(oracle):
    """CPU pin: the edge cases above are ones where merge-then-encode is not decode-then-encode
    (so the GPU test below checks the documented semantics, not a coincidence)."""
    differ = 0
    for u in edge_updates():
        code, merged = oracle.status_of(oracle.merge_updates_v1, [u])
        assert code == 0
        direct = oracle.merge_updates_v2([u], inputs_v1=True)
        assert direct == oracle.convert_update_v1_to_v2(merged)  # single-client DeleteSets: no order question
        differ += direct != oracle.convert_update_v1_to_v2(u)
    assert differ >= 3


@pytest.mark.gpu
def test_convert_v1_to_v2_device_merge_semantics(oracle):
    """Overlapping same-client blocks and adjacent Skips: the entry is merge-then-encode."""
    import numpy as np
    import ymerge
    ups = edge_updates()
    data = np.frombuffer(b"".join(ups), np.uint8).copy()
    offs = np.concatenate([[0], np.cumsum([len(u) for u in ups])]).astype(np.uint64)
    e = ymerge.Engine(0)
    try:
        out, off, st = e.convert_v1_to_v2_host(data, offs)
    finally:
        e.close()
    for i, u in enumerate(ups):
        code, merged = oracle.status_of(oracle.merge_updates_v1, [u])
        assert int(st[i]) == code, (i, int(st[i]), code)
        if code == 0:
            want = oracle.merge_updates_v2([u], inputs_v1=True)
            assert out[int(off[i]):int(off[i + 1])].tobytes() == want, i


@pytest.mark.gpu
def test_edge_updates_merge_sv_diff(oracle):
    """The same edge updates through merge_updates_v1 (each alone and all in one document),
    the state vector and diff_updates_v1 against an empty state vector: a client repeated in a
    later section (update 1: its blocks queue in section order, REC_ORDER) must follow yrs'
    queue order on every path, not the clock order the sort-based paths use."""
    import numpy as np
    import ymerge
    ups = edge_updates()
    e = ymerge.Engine(0)
    try:
        for docs in ([[u] for u in ups], [ups], [[ups[1], ups[0], ups[2]]]):
            data = np.frombuffer(b"".join(b"".join(d) for d in docs), np.uint8).copy()
            lens = [len(u) for d in docs for u in d]
            upd_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
            doc_upd = np.concatenate([[0], np.cumsum([len(d) for d in docs])]).astype(np.uint64)
            out, off, st = e.merge_host(data, upd_off, doc_upd)
            for k, d in enumerate(docs):
                code, want = oracle.status_of(oracle.merge_updates_v1, d)
                assert int(st[k]) == code, (k, int(st[k]), code)
                if code == 0:
                    assert out[int(off[k]):int(off[k + 1])].tobytes() == want, k
        data = np.frombuffer(b"".join(ups), np.uint8).copy()
        u_off = np.concatenate([[0], np.cumsum([len(u) for u in ups])]).astype(np.uint64)
        sv, sv_off, sv_st = e.state_vector_host(data, u_off)
        empty = np.zeros(len(ups), np.uint8)
        df, df_off, df_st = e.diff_host(data, u_off, empty, np.arange(len(ups) + 1, dtype=np.uint64))
    finally:
        e.close()
    for i, u in enumerate(ups):
        code, want = oracle.status_of(oracle.encode_state_vector_from_update_v1, u)
        assert int(sv_st[i]) == code, ("sv", i, int(sv_st[i]), code)
        if code == 0:
            assert sv[int(sv_off[i]):int(sv_off[i + 1])].tobytes() == want, ("sv", i)
        code, want = oracle.status_of(oracle.diff_updates_v1, u, b"\x00")
        assert int(df_st[i]) == code, ("diff", i, int(df_st[i]), code)
        if code == 0:
            assert df[int(df_off[i]):int(df_off[i + 1])].tobytes() == want, ("diff", i)
