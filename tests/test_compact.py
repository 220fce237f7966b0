"""Store-based compaction oracle (oracle/yrs_oracle_store.c: a yrs Doc with GC on applies a
document's updates in order, one transaction each, then encode_state_as_update_v1), pinned on:

* the offline Yjs bundle (tools/yjs/check_compact.py -> tests/golden/compact_yjs_check.json):
  Yjs implements the same integration, GC and struct merging; its encodeStateAsUpdate is
  byte-identical to the oracle on the five editing traces (259,778 updates for
  automerge-paper, text == endContent), on in-order scenario fixtures and on the reference's
  merge_pending_updates test (yrs/src/update.rs:1269-1333, text "nenor");
* the reference's KATs (yrs/src/alt.rs:103-160, compatibility_tests.rs payloads) and its
  update_merge property (update.rs:1125-1164: the order of the updates and a prior merge do
  not change the compacted state).

Documented divergences from Yjs (the oracle follows yrs): DeleteSet client order (hash order,
Yjs sorts), Any numbers, a String split inside a surrogate pair (yrs keeps the pair,
block.rs:1483-1502), and a DeleteSet for a client with no blocks yet, which yrs' apply_delete
drops instead of keeping pending (transaction.rs:474-476)."""
import hashlib
import json
import os

import pytest

from conftest import ROOT
from test_oracle_kats import ALT_MERGE_1, ALT_MERGE_2, COMPAT

GOLD = os.path.join(ROOT, "tests", "golden")
# fixtures whose Yjs bytes differ, and why (see the module docstring)
DIVERGE = {
    "single_typing_60_rev": "ds_unknown_client", "single_typing_60_shuf": "ds_unknown_client",
    "single_typing_150_rev": "ds_unknown_client", "single_typing_150_shuf": "ds_unknown_client",
    "synced_3clients": "ds_order", "concurrent_2": "ds_order", "numbers": "any_numbers",
    "utf16_text": "surrogate_split", "utf16_log_then_snapshot": "surrogate_split",
}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def var(x):
    out = bytearray()
    while True:
        b, x = x & 0x7F, x >> 7
        out.append(b | (0x80 if x else 0))
        if not x:
            return bytes(out)


def vstr(s):
    b = s.encode()
    return var(len(b)) + b


@pytest.fixture(scope="module")
def check():
    with open(os.path.join(GOLD, "compact_yjs_check.json")) as f:
        return json.load(f)["cases"]


def test_kats(oracle):
    for a, b, exp in (ALT_MERGE_1, ALT_MERGE_2):
        assert list(oracle.compact_updates_v1([bytes(a), bytes(b)])) == exp
        assert list(oracle.compact_updates_v1([bytes(b), bytes(a)])) == exp
    for u in COMPAT.values():  # states encoded by yrs re-encode to themselves
        assert oracle.compact_updates_v1([bytes(u)]) == bytes(u)
        assert oracle.compact_updates_v1([bytes(u), bytes(u)]) == bytes(u)


def test_update_merge_property(oracle):
    """update.rs:1125-1164: client 1 inserts "aaa" twice at 0, client 2 inserts "bbb" at 0 and
    "bbb" at 2 (one transaction each); applying the two updates in either order, or their
    merge, gives the same compacted state."""
    t = var(1) + vstr("test")
    b1 = var(1) + var(2) + var(1) + var(0) + bytes([0x04]) + t + vstr("aaa") + bytes([0x44]) + var(1) + var(0) + \
        vstr("aaa") + var(0)
    b2 = var(1) + var(3) + var(2) + var(0) + bytes([0x04]) + t + vstr("bb") + bytes([0x84]) + var(2) + var(1) + \
        vstr("b") + bytes([0xC4]) + var(2) + var(1) + var(2) + var(2) + vstr("bbb") + var(0)
    c12 = oracle.compact_updates_v1([b1, b2])
    assert oracle.compact_updates_v1([b2, b1]) == c12
    assert oracle.compact_updates_v1([oracle.merge_updates_v1([b1, b2], mode=1)]) == c12
    assert oracle.compact_updates_v1([c12]) == c12


def test_yjs_traces(oracle, check):
    import workloads
    rows = {c["name"]: c for c in check if c["kind"] == "trace"}
    assert len(rows) == len(workloads.TRACES)
    for name in workloads.TRACES:
        b, _ = workloads.trace_updates(name)
        c = oracle.compact_updates_v1(b.doc_updates(0))
        r = rows[name]
        assert r["byte_equal"] and r["text_equal"], r
        assert sha(c) == r["compact_sha256"] == r["yjs_sha256"], name


def test_yjs_fixtures(oracle, check):
    with open(os.path.join(GOLD, "yjs_fixtures.json")) as f:
        cases = {c["name"]: c for c in json.load(f)["cases"]}
    rows = [c for c in check if c["kind"] == "fixture"]
    assert len(rows) >= 35
    for r in rows:
        c = oracle.compact_updates_v1([bytes.fromhex(h) for h in cases[r["name"]]["updates"]])
        assert sha(c) == r["compact_sha256"], r["name"]
        why = DIVERGE.get(r["name"])
        if why is None:
            assert r["byte_equal"] and r["compact_sha256"] == r["yjs_sha256"], r
        elif why == "ds_order":
            assert r["content_equal"], r


def test_merge_pending_updates(oracle, check):
    """update.rs:1269-1333 restated: the chain of documents re-encoding their state, with
    updates[3] (pending: clock 2 missing) before updates[2]."""
    def up(clock, ch):
        blk = (bytes([0x04]) + var(1) + vstr("textBlock") if clock == 0
               else bytes([0x44]) + var(0) + var(clock - 1)) + vstr(ch)
        return var(1) + var(1) + var(0) + var(clock) + blk + var(0)
    u = [up(k, ch) for k, ch in enumerate("ronen")]
    c1 = oracle.compact_updates_v1([u[0]])
    c2 = oracle.compact_updates_v1([c1, u[1]])
    c3 = oracle.compact_updates_v1([c2, u[3]])
    c4 = oracle.compact_updates_v1([c3, u[2]])
    c5 = oracle.compact_updates_v1([c4, u[4]])
    r = next(c for c in check if c["kind"] == "merge_pending_updates")
    assert r["text_equal"] and r["byte_equal"]
    assert sha(c5) == r["compact_sha256"]
    # the pending block (clock 3) travels inside c3 until clock 2 arrives
    assert len(c3) > len(c2)


def test_errors(oracle):
    assert oracle.status_of(oracle.compact_updates_v1, [b""])[0] == 3
    move = var(1) + var(1) + var(5) + var(0) + bytes([0x0B]) + var(1) + vstr("t") + var(1) + var(5) + var(0) + var(0)
    assert oracle.status_of(oracle.compact_updates_v1, [move])[0] == 21  # Move content: not restated
