"""TEST TOOLING ONLY (this container): pins the store-based compaction oracle
(oracle/yrs_oracle_store.c) on the offline Yjs bundle.

Yjs implements the same YATA integration, GC and struct merging as yrs (yrs is its port);
per case a fresh Y.Doc applies the updates in order and encodes its state
(Y.encodeStateAsUpdate).  Recorded per case: the oracle's compaction sha256, whether Yjs's
bytes are identical, whether the two documents hold the same content (Yjs applying the
oracle's bytes), and for the editing traces whether the text equals the trace's endContent.
Cases: the five editing traces (one update per patch) and the Yjs scenario fixtures.
Writes tests/golden/compact_yjs_check.json.

    python tools/yjs/check_compact.py
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
import oracle  # noqa: E402
import workloads  # noqa: E402


def sha(b):
    return hashlib.sha256(b).hexdigest()


def var(x):
    out = bytearray()
    while True:
        b, x = x & 0x7F, x >> 7
        out.append(b | (0x80 if x else 0))
        if not x:
            return bytes(out)


def pending_updates():
    ups = []
    for clock, ch in enumerate("rone" + "n"):
        if clock == 0:
            blk = bytes([0x04]) + var(1) + var(9) + b"textBlock" + var(1) + ch.encode()
        else:  # inserted at index 0: right origin = the previous first character
            blk = bytes([0x44]) + var(0) + var(clock - 1) + var(1) + ch.encode()
        ups.append(var(1) + var(1) + var(0) + var(clock) + blk + var(0))
    return ups


def pending_chain():
    u = pending_updates()
    c1 = oracle.compact_updates_v1([u[0]])
    c2 = oracle.compact_updates_v1([c1, u[1]])
    c3 = oracle.compact_updates_v1([c2, u[3]])
    c4 = oracle.compact_updates_v1([c3, u[2]])
    c5 = oracle.compact_updates_v1([c4, u[4]])
    return [c1, c2, c3, c4, c5]


def main():
    oracle.build()
    names, rows = [], []
    for name in workloads.TRACES:
        b, end = workloads.trace_updates(name)
        ups = b.doc_updates(0)
        c = oracle.compact_updates_v1(ups)
        names.append(("trace", name, len(ups)))
        rows.append({"updates": [u.hex() for u in ups], "compact": c.hex(), "end": end})
        print(name, len(ups), len(c), flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "yjs_fixtures.json")) as f:
        cases = json.load(f)["cases"]
    for i, cs in enumerate(cases):
        ups = [bytes.fromhex(h) for h in cs["updates"]]
        st, c = oracle.status_of(oracle.compact_updates_v1, ups)
        if st:
            print("fixture", i, "status", st)
            continue
        names.append(("fixture", cs.get("name", str(i)), len(ups)))
        rows.append({"updates": cs["updates"], "compact": c.hex()})
    # yrs/src/update.rs:1269-1333 (merge_pending_updates): five one-char inserts at index 0 of
    # "textBlock" by client 0, re-encoded through a chain of documents with updates[3] before
    # updates[2] (pending structs); the last document's text must be "nenor"
    chain = pending_chain()
    names.append(("merge_pending_updates", "update.rs:1269-1333", 5))
    rows.append({"updates": [chain[-1].hex()], "compact": chain[-1].hex(), "root": "textBlock", "end": "nenor"})
    tmp = "/tmp/ymerge_compact_check.json"
    with open(tmp, "w") as f:
        json.dump(rows, f)
    js = os.path.join(os.path.dirname(os.path.abspath(__file__)), "check_compact.js")
    res = json.loads(subprocess.check_output(["node", "--max-old-space-size=8192", js, tmp]))
    out = []
    for (kind, name, n), row, r in zip(names, rows, res):
        c = bytes.fromhex(row["compact"])
        e = {"kind": kind, "name": name, "updates": n, "compact_len": len(c), "compact_sha256": sha(c),
             "yjs_sha256": sha(bytes.fromhex(r["yjs_hex"])), "byte_equal": r["byte_equal"],
             "content_equal": r["content_equal"]}
        if "text_equal" in r:
            e["text_equal"] = r["text_equal"]
        if "error" in r:
            e["yjs_error"] = r["error"]
        out.append(e)
        print(kind, name, {k: v for k, v in e.items() if k.endswith("equal")})
    with open(os.path.join(ROOT, "tests", "golden", "compact_yjs_check.json"), "w") as f:
        json.dump({"check": "Yjs: fresh Y.Doc, applyUpdate per update in order, encodeStateAsUpdate; "
                            "oracle: yo_compact_updates_v1",
                   "cases": out}, f, indent=1)


if __name__ == "__main__":
    main()
