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
    "subdoc": None,  # subdoc: the oracle reports UNSUPPORTED too
    # rich_text (Format / Embed items), map_array_any, map_array_xml_nested and numbers (maps,
    # nested types, Any content) are on the device since round 6
}


def fixture_reason(name):
    for k, v in FIXTURE_REASONS.items():
        if name.endswith(k) if k.startswith("_") else name == k:
            return v
    return 0


def edge_docs():
    """Small hand-built documents: empty, malformed, KAT-style, 10 / 16 / 17 clients, a split inside a
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
    # ten clients (on the device since round 6), sixteen (the most), seventeen (refused)
    for ncl, why in ((10, 0), (16, 0), (17, CU["CLIENTS"])):
        ups = [upd(1, 0, [s_root("a")])]
        for c in range(2, ncl + 1):
            ups.append(upd(c, 0, [s_after(c - 1, 0, "x")]))
        docs.append(ups); reasons.append(why)
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
    # map entry (parent_sub) with a String value
    docs.append([upd(1, 0, [bytes([0x24]) + t + vstr("k") + vstr("v")])]); reasons.append(0)
    docs += nested_docs()
    reasons += [0] * (len(docs) - len(reasons) - 1) + [None]
    return batch_of(docs), reasons


def _anys(vals):
    """ItemContent::Any (ref 8): strings (tag 119), ints (125), null (126)."""
    b = var(len(vals))
    for v in vals:
        if v is None:
            b += bytes([126])
        elif isinstance(v, int):
            b += bytes([125]) + var(2 * v)  # (non-negative: the sign bit 6 clear; v < 64)
        else:
            b += bytes([119]) + vstr(v)
    return b


def nested_docs():
    """Maps, nested types and list contents (round 6): a key written twice, concurrent writes of
    one key from two clients in both delivery orders, a nested array with Any items squashed,
    split by a delete and then deleted with its type (children become GC structs), XmlElement
    / XmlText nesting, a JSON list split by a delete, and (last) an ID parent that is not a
    type (yrs panics)."""
    t = var(1) + vstr("t")

    def upd(client, clock, blocks, ds=b"\x00"):
        return var(1) + var(len(blocks)) + var(client) + var(clock) + b"".join(blocks) + ds

    def dsu(client, ranges):
        return b"\x00" + var(1) + var(client) + var(len(ranges)) + b"".join(var(a) + var(n) for a, n in ranges)

    def idp(c, k):
        return var(0) + var(c) + var(k)

    docs = []
    # a key written twice: the second value (origin = the first) deletes the first
    docs.append([upd(1, 0, [bytes([0x28]) + t + vstr("k") + _anys(["a"])]),
                 upd(1, 1, [bytes([0x88]) + var(1) + var(0) + _anys(["b", 7])])])
    # two clients write the same key concurrently (no origins): both delivery orders
    k1 = upd(1, 0, [bytes([0x28]) + t + vstr("k") + _anys(["one"])])
    k2 = upd(2, 0, [bytes([0x28]) + t + vstr("k") + _anys(["two"])])
    docs.append([k1, k2])
    docs.append([k2, k1])
    # a nested array under a map key; Any items appended (squashed), one element deleted (split),
    # then the array deleted: its children become GC structs
    arr = upd(1, 0, [bytes([0x27]) + t + vstr("arr") + bytes([0])])
    c1 = upd(1, 1, [bytes([0x08]) + idp(1, 0) + _anys([1, 2, 3])])
    c2 = upd(1, 4, [bytes([0x88]) + var(1) + var(3) + _anys([4, None])])
    docs.append([arr, c1, c2])
    docs.append([arr, c1, c2, dsu(1, [(2, 1)])])
    docs.append([arr, c1, c2, dsu(1, [(2, 1)]), dsu(1, [(0, 1)])])
    docs.append([arr, c1, c2, dsu(1, [(0, 1)])])
    # XmlElement "p" in root "x", an XmlText in it, a String in that; a second client types after it
    x = var(1) + vstr("x")
    e1 = upd(1, 0, [bytes([0x07]) + x + bytes([3]) + vstr("p")])
    e2 = upd(1, 1, [bytes([0x07]) + idp(1, 0) + bytes([6])])
    e3 = upd(1, 2, [bytes([0x04]) + idp(1, 1) + vstr("hi")])
    e4 = upd(2, 0, [bytes([0x84]) + var(1) + var(3) + vstr("!")])
    docs.append([e1, e2, e3, e4])
    docs.append([e1, e2, e3, e4, dsu(1, [(3, 1)]), dsu(1, [(1, 1)])])
    # a JSON list (ref 2: L + 1 JSON texts) split by deleting its middle element
    j = upd(1, 0, [bytes([0x02]) + t + var(2) + vstr('"a"') + vstr("1") + vstr("null")])
    docs.append([j, dsu(1, [(1, 1)])])
    # an ID parent that is a String item: "parent points to a block which is not a shared type"
    docs.append([upd(1, 0, [bytes([0x04]) + t + vstr("ab")]), upd(1, 2, [bytes([0x04]) + idp(1, 0) + vstr("z")])])
    return docs


# ---------------------------------------------------------------- an independent shape check
# A plain restatement of the lib0 v1 grammar (yrs/src/update.rs:433-488, 714-749) used to
# confirm, from the bytes alone, the reason the device gives for refusing a document (the
# status comparison against tools/hostemu is the same kernel source; this is not).

def _rv(b, i):
    r = s = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7F) << s
        s += 7
        if x < 0x80:
            return r, i


def _str(b, i):
    n, i = _rv(b, i)
    return b[i:i + n], i + n


def _any(b, i):
    t = b[i]
    i += 1
    if t in (127, 126, 121, 120):
        return i
    if t == 125:
        return _rv(b, i)[1]
    if t == 124:
        return i + 4
    if t in (123, 122):
        return i + 8
    if t in (119, 116):
        return _str(b, i)[1]
    if t == 118:
        n, i = _rv(b, i)
        for _ in range(n):
            i = _any(b, _str(b, i)[1])
        return i
    if t == 117:
        n, i = _rv(b, i)
        for _ in range(n):
            i = _any(b, i)
        return i
    raise ValueError(t)


def parse_v1(u):
    """(blocks, ds): blocks as dicts (client, clock, len, ref, skip, origin, rorigin, id_parent,
    psub); ds as [(client, [(start, len)])].  Raises on malformed input."""
    b = bytes(u)
    blocks, ds = [], []
    ncl, i = _rv(b, 0)
    for _ in range(ncl):
        nb, i = _rv(b, i)
        client, i = _rv(b, i)
        clock, i = _rv(b, i)
        for _ in range(nb):
            info = b[i]
            i += 1
            blk = dict(client=client, clock=clock, ref=info & 15, skip=info == 10, gc=info == 0, origin=None,
                       rorigin=None, id_parent=None, psub=False)
            if info in (0, 10):
                ln, i = _rv(b, i)
            else:
                if info & 0x80:
                    oc, i = _rv(b, i)
                    ok, i = _rv(b, i)
                    blk["origin"] = (oc, ok)
                if info & 0x40:
                    rc, i = _rv(b, i)
                    rk, i = _rv(b, i)
                    blk["rorigin"] = (rc, rk)
                if info & 0xC0 == 0:
                    pi, i = _rv(b, i)
                    if pi == 1:
                        i = _str(b, i)[1]
                    else:
                        pc, i = _rv(b, i)
                        pk, i = _rv(b, i)
                        blk["id_parent"] = (pc, pk)
                    if info & 0x20:
                        blk["psub"] = True
                        i = _str(b, i)[1]
                ref = info & 15
                if ref == 1:
                    ln, i = _rv(b, i)
                elif ref == 4:
                    s, i = _str(b, i)
                    ln = len(s.decode("utf-8", "surrogatepass").encode("utf-16-le")) // 2
                elif ref == 2:
                    n, i = _rv(b, i)
                    for _ in range(n + 1):
                        i = _str(b, i)[1]
                    ln = n + 1
                elif ref in (3, 5):
                    i = _str(b, i)[1]
                    ln = 1
                elif ref == 6:
                    i = _str(b, _str(b, i)[1])[1]
                    ln = 1
                elif ref == 7:
                    tr = b[i]
                    i += 1
                    if tr == 3:
                        i = _str(b, i)[1]
                    ln = 1
                elif ref == 8:
                    n, i = _rv(b, i)
                    for _ in range(n):
                        i = _any(b, i)
                    ln = n
                elif ref == 9:
                    i = _any(b, _str(b, i)[1])
                    ln = 1
                else:
                    raise ValueError(ref)
            blk["len"] = ln
            blocks.append(blk)
            clock += ln
    ne, i = _rv(b, i)
    for _ in range(ne):
        c, i = _rv(b, i)
        nr, i = _rv(b, i)
        rs = []
        for _ in range(nr):
            s, i = _rv(b, i)
            ln, i = _rv(b, i)
            rs.append((s, ln))
        ds.append((c, rs))
    return blocks, ds


def exhibits(updates, reason):
    """True when the document's bytes show the shape `reason` (a CU code) names, False when they
    do not, None for the capacity reasons (scratch sizes) a byte-level check cannot restate."""
    try:
        parsed = [parse_v1(u) for u in updates]
    except (ValueError, IndexError):
        return None
    if reason == CU["CLIENTS"]:
        cls = {b["client"] for bl, _ in parsed for b in bl}
        cls_ds = cls | {c for _, ds in parsed for c, _ in ds}
        return len(cls) > 16 or len(cls_ds) > 16  # ycompact.hip CP_MAXCL
    if reason == CU["PARENT"]:
        return any(b["id_parent"] is not None or b["psub"] for bl, _ in parsed for b in bl)
    if reason == CU["UPDATE_SHAPE"]:
        return any(not b["gc"] and not b["skip"] and b["ref"] not in (1, 3, 4, 5, 6) for bl, _ in parsed for b in bl) or \
            any(len(ds) > 16 for _, ds in parsed)
    if reason in (CU["GAP"], CU["PENDING"], CU["PENDING_DS"]):
        nxt, gap, pend, pds = {}, False, False, False
        for bl, ds in parsed:
            for b in bl:
                if b["skip"]:
                    gap = True
                    continue
                c = b["client"]
                if b["clock"] > nxt.get(c, 0):
                    gap = True
                    continue
                for dep in (b["origin"], b["rorigin"], b["id_parent"]):
                    if dep is not None and dep[1] >= nxt.get(dep[0], 0) and dep[0] != c:
                        pend = True
                    if dep is not None and dep[0] == c and dep[1] >= b["clock"] and b["clock"] >= nxt.get(c, 0):
                        pend = True
                nxt[c] = max(nxt.get(c, 0), b["clock"] + b["len"])
            for c, rs in ds:
                for s, ln in rs:
                    if c in nxt and s + ln > nxt[c]:
                        pds = True
        return gap or pend or pds  # (delivery out of order shows as any of the three)
    return None
