"""Pins the CPU oracle against the reference's own byte-exact vectors.

yrs/src/alt.rs:103-160 (4 KATs), yrs/src/tests/compatibility_tests.rs (v1
payloads + the hashbrown-collision state vector at :293-318) and
yrs/src/update.rs:1083-1122 (map update decode).
"""
import json
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

ALT_MERGE_1 = (
    [1, 1, 220, 240, 237, 172, 15, 0, 4, 1, 4, 116, 101, 115, 116, 3, 97, 98, 99, 0],
    [1, 1, 201, 139, 250, 201, 1, 0, 4, 1, 4, 116, 101, 115, 116, 2, 100, 101, 0],
    [2, 1, 220, 240, 237, 172, 15, 0, 4, 1, 4, 116, 101, 115, 116, 3, 97, 98, 99, 1, 201,
     139, 250, 201, 1, 0, 4, 1, 4, 116, 101, 115, 116, 2, 100, 101, 0],
)
ALT_MERGE_2 = (
    [1, 1, 129, 231, 135, 164, 7, 0, 4, 1, 4, 49, 50, 51, 52, 1, 97, 0],
    [1, 1, 129, 231, 135, 164, 7, 1, 68, 129, 231, 135, 164, 7, 0, 1, 98, 0],
    [1, 2, 129, 231, 135, 164, 7, 0, 4, 1, 4, 49, 50, 51, 52, 1, 97, 68, 129, 231, 135, 164,
     7, 0, 1, 98, 0],
)
ALT_SV = (
    [2, 1, 220, 240, 237, 172, 15, 0, 4, 1, 4, 116, 101, 115, 116, 3, 97, 98, 99, 1, 201,
     139, 250, 201, 1, 0, 4, 1, 4, 116, 101, 115, 116, 2, 100, 101, 0],
    [2, 220, 240, 237, 172, 15, 3, 201, 139, 250, 201, 1, 2],
)
ALT_DIFF = (
    [1, 2, 148, 189, 145, 162, 9, 0, 4, 1, 4, 116, 101, 115, 116, 3, 97, 98, 99, 68, 148,
     189, 145, 162, 9, 0, 2, 100, 101, 0],
    [1, 148, 189, 145, 162, 9, 3],
    [1, 1, 148, 189, 145, 162, 9, 3, 68, 148, 189, 145, 162, 9, 0, 2, 100, 101, 0],
)
# canonical single updates: merge([u]) == u, diff(u, {}) == u
COMPAT = {
    "text_insert_delete": [1, 5, 152, 234, 173, 126, 0, 1, 1, 4, 116, 121, 112, 101, 3, 68, 152,
                           234, 173, 126, 0, 2, 97, 98, 193, 152, 234, 173, 126, 4, 152, 234,
                           173, 126, 0, 1, 129, 152, 234, 173, 126, 2, 1, 132, 152, 234, 173,
                           126, 6, 2, 104, 105, 1, 152, 234, 173, 126, 2, 0, 3, 5, 2],
    "map_set": [1, 2, 241, 204, 241, 209, 1, 0, 40, 1, 4, 116, 101, 115, 116, 2, 107, 49, 1,
                119, 2, 118, 49, 40, 1, 4, 116, 101, 115, 116, 2, 107, 50, 1, 119, 2, 118, 50, 0],
    "array_insert": [1, 1, 208, 180, 170, 180, 9, 0, 8, 1, 4, 116, 101, 115, 116, 2, 119, 1, 97,
                     119, 1, 98, 0],
    "xml_fragment_insert": [1, 2, 144, 163, 251, 148, 9, 0, 7, 1, 13, 102, 114, 97, 103, 109,
                            101, 110, 116, 45, 110, 97, 109, 101, 6, 135, 144, 163, 251, 148, 9,
                            0, 3, 9, 110, 111, 100, 101, 45, 110, 97, 109, 101, 0],
    "update_decode": [1, 1, 176, 249, 159, 198, 7, 0, 40, 1, 0, 4, 107, 101, 121, 66, 1, 119, 6,
                      118, 97, 108, 117, 101, 66, 0],
}
SV_COLLISION = [2, 178, 219, 218, 44, 3, 190, 212, 225, 6, 2]


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("kat", [ALT_MERGE_1, ALT_MERGE_2])
def test_alt_merge(oracle, kat, mode):
    a, b, exp = kat
    assert list(oracle.merge_updates_v1([bytes(a), bytes(b)], mode)) == exp


def test_alt_sv(oracle):
    u, exp = ALT_SV
    assert list(oracle.encode_state_vector_from_update_v1(bytes(u))) == exp


def test_alt_diff(oracle):
    u, sv, exp = ALT_DIFF
    assert list(oracle.diff_updates_v1(bytes(u), bytes(sv))) == exp


@pytest.mark.parametrize("name", sorted(COMPAT))
def test_compat_roundtrip(oracle, name):
    u = bytes(COMPAT[name])
    assert oracle.merge_updates_v1([u], 0) == u
    assert oracle.merge_updates_v1([u, u], 1) == u  # duplicates collapse (update.rs:1167-1180)
    assert oracle.diff_updates_v1(u, b"\x00") == u


def test_sv_hash_collision_order(oracle):
    # 93760946 & 3 == 14182974 & 3 == 2: second key probes to slot 3
    assert list(oracle.sv_roundtrip(bytes(SV_COLLISION))) == SV_COLLISION


def test_merge_idempotent(oracle):
    # update.rs:1183-1207: merge of a merge is stable
    a, b, _ = ALT_MERGE_1
    m = oracle.merge_updates_v1([bytes(a), bytes(b)])
    assert oracle.merge_updates_v1([m]) == m


def test_empty_and_errors(oracle):
    assert oracle.merge_updates_v1([]) == bytes([0, 0])
    assert oracle.merge_updates_v1([bytes([0, 0])]) == bytes([0, 0])
    st, _ = oracle.status_of(oracle.merge_updates_v1, [b""])
    assert st == 3  # EndOfBuffer
    st, _ = oracle.status_of(oracle.merge_updates_v1, [bytes([0x80] * 12)])
    assert st == 2  # InvalidVarInt
    # content ref 12 -> UnexpectedValue
    st, _ = oracle.status_of(oracle.merge_updates_v1, [bytes([1, 1, 5, 0, 0x0C, 1, 0])])
    assert st == 4
    # first failing update wins
    st, _ = oracle.status_of(oracle.merge_updates_v1, [bytes([1, 1, 5, 0, 0x0C, 1, 0]), b""])
    assert st == 4


def _fixtures():
    with open(os.path.join(HERE, "golden", "yjs_fixtures.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", _fixtures(), ids=lambda c: c["name"])
def test_yjs_crosscheck(oracle, case):
    """Byte-equality with Yjs where yrs and Yjs provably agree;
    equality modulo DeleteSet client order for multi-client text cases."""
    ups = [bytes.fromhex(h) for h in case["updates"]]
    st, m = oracle.status_of(oracle.merge_updates_v1, ups, 0)
    assert st == 0
    if case["name"] == "rich_text":  # Format/Embed JSON round trip: single-key objects, so byte-equal
        assert m == bytes.fromhex(case["yjs_merge"])
    assert oracle.merge_updates_v1(ups, 1) == m
    y = bytes.fromhex(case["yjs_merge"])
    if case["agree"]:
        assert m == y
        assert oracle.encode_state_vector_from_update_v1(m).hex() == case["yjs_sv"]
        for d in case["diffs"]:
            assert oracle.diff_updates_v1(y, bytes.fromhex(d["sv"])).hex() == d["yjs"]
    elif case["name"].startswith(("synced", "concurrent")):
        assert oracle.normalized(m) == oracle.normalized(y)
        assert sorted(oracle.parse_sv(oracle.encode_state_vector_from_update_v1(m))) == \
            sorted(oracle.parse_sv(bytes.fromhex(case["yjs_sv"])))
