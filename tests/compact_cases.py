"""Batches for the store-based compaction parity tests (tests/test_compact_emu.py on the CPU,
tests/test_gpu_compact.py on the MI355X), with the device-shape reason (ycompact.hip CU_*)
each unsupported document is expected to carry."""
import json
import os

import numpy as np

import workloads
from conftest import ROOT

# ycompact.hip CU_* codes
CU = dict(CLIENTS=1, ITEMS=2, SURROGATE=3, TXN=4, ARRIVALS=5, GAP=6, PARTIAL=7, PARENT=8, ROOTS=9,
          PENDING_DS=10, PENDING=11, UPDATE_SHAPE=12, OUTPUT=13)


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


def batch_of(docs):
    parts, offs, dus, tot = [], [0], [0], 0
    for ups in docs:
        for u in ups:
            parts.append(np.frombuffer(bytes(u), dtype=np.uint8))
            tot += len(u)
            offs.append(tot)
        dus.append(len(offs) - 1)
    data = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return workloads.Batch(data, np.array(offs, np.uint64), np.array(dus, np.uint64))


def regrouped(oracle, b, k=None, head=None):
    """Each document's updates merged k at a time (multi-client updates: the dependency
    stack), or its first `head` updates merged into one snapshot followed by the rest."""
    docs = []
    for d in range(b.n_docs):
        u = b.doc_updates(d)
        if k:
            docs.append([oracle.merge_updates_v1(u[i:i + k], mode=1) for i in range(0, len(u), k)])
        else:
            docs.append([oracle.merge_updates_v1(u[:head], mode=1)] + list(u[head:]))
    return batch_of(docs)


def fixtures():
    """tests/golden/yjs_fixtures.json (Yjs-generated update logs): one document each."""
    with open(os.path.join(ROOT, "tests", "golden", "yjs_fixtures.json")) as f:
        cases = json.load(f)["cases"]
    return [c["name"] for c in cases], batch_of([[bytes.fromhex(h) for h in c["updates"]] for c in cases])


# fixtures outside the device shape and why (everything else must be written by the device)
FIXTURE_REASONS = {
    "_rev": CU["GAP"], "_shuf": CU["GAP"],  # out-of-order delivery: pending structs
    "utf16_text": CU["SURROGATE"], "utf16_log_then_snapshot": CU["SURROGATE"],
    "map_array_any": CU["UPDATE_SHAPE"], "map_array_xml_nested": CU["UPDATE_SHAPE"], "numbers": CU["UPDATE_SHAPE"],
    "rich_text": CU["UPDATE_SHAPE"], "subdoc": None,  # subdoc: the oracle reports UNSUPPORTED too
}


def fixture_reason(name):
    for k, v in FIXTURE_REASONS.items():
        if name.endswith(k) if k.startswith("_") else name == k:
            return v
    return 0


def edge_docs():
    """Small hand-built documents: empty, malformed, KAT-style, nine clients, a split inside a
    surrogate pair, a Skip block, a delete of a client the store has never seen."""
    t = var(1) + vstr("t")

    def upd(client, clock, blocks, ds=b"\x00"):
        return var(1) + var(len(blocks)) + var(client) + var(clock) + b"".join(blocks) + ds

    def s_root(text):
        return bytes([0x04]) + t + vstr(text)

    def s_after(oc, ok, text):
        return bytes([0x84]) + var(oc) + var(ok) + vstr(text)

    docs, reasons = [], []
    docs.append([]); reasons.append(0)                                   # no updates: empty Doc
    docs.append([b""]); reasons.append(None)                             # EOS (decode error)
    docs.append([b"\x00\x00"]); reasons.append(0)                        # empty update
    docs.append([upd(1, 0, [s_root("abc")]), upd(1, 3, [s_after(1, 2, "def")])]); reasons.append(0)
    # deleting inside an item: split + merge_blocks + GC squash
    docs.append([upd(1, 0, [s_root("hello world")]),
                 b"\x00" + var(1) + var(1) + var(1) + var(2) + var(5)]); reasons.append(0)
    # a delete set for a client with no blocks: dropped (transaction.rs:474-476)
    docs.append([upd(1, 0, [s_root("ab")]), b"\x00" + var(1) + var(9) + var(1) + var(0) + var(1)]); reasons.append(0)
    # nine clients
    ups = [upd(1, 0, [s_root("a")])]
    for c in range(2, 11):
        ups.append(upd(c, 0, [s_after(c - 1, 0, "x")]))
    docs.append(ups); reasons.append(CU["CLIENTS"])
    # a split inside a surrogate pair (yrs keeps the pair on the left)
    docs.append([upd(1, 0, [s_root("a\U0001F600b")]), upd(2, 0, [s_after(1, 1, "z")])]); reasons.append(CU["SURROGATE"])
    # Skip block inside an update
    docs.append([upd(1, 0, [s_root("ab")]), upd(1, 2, [bytes([10]) + var(3), s_after(1, 4, "q")])]); reasons.append(CU["GAP"])
    # clock gap (pending)
    docs.append([upd(1, 0, [s_root("ab")]), upd(1, 5, [s_after(1, 4, "q")])]); reasons.append(CU["GAP"])
    # duplicate delivery (fully known blocks are skipped)
    u0 = upd(1, 0, [s_root("abc")])
    docs.append([u0, u0, upd(1, 3, [s_after(1, 2, "d")]), u0]); reasons.append(0)
    # GC block then items
    docs.append([upd(1, 0, [b"\x00" + var(4)]), upd(1, 4, [s_after(1, 3, "x")])]); reasons.append(0)
    # map entry (parent_sub): outside the shape
    docs.append([upd(1, 0, [bytes([0x24]) + t + vstr("k") + vstr("v")])]); reasons.append(CU["PARENT"])
    return batch_of(docs), reasons
