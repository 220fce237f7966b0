"""TEST TOOLING ONLY (this container): pins the oracle on the reference's editing traces.

For each trace of assets/editing-traces/sequential_traces (copied to tests/golden/) the
trace is replayed as one v1 update per patch (workloads.trace_updates), the CPU oracle
merges all of them (merge_updates_v1), and the offline Yjs bundle applies the merge to a
fresh Y.Doc: its "text" must equal the trace's endContent.  The diff path is checked
the same way: Yjs applies the merge of the first half of the updates, then
diff_updates_v1(full merge, state vector of that half merge), and must again reach
endContent.  Writes tests/golden/traces_yjs_check.json (sha256 of every result).

    python tools/yjs/check_traces.py
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


def main():
    rows, fx = [], {}
    for name in workloads.TRACES:
        b, end = workloads.trace_updates(name)
        ups = b.doc_updates(0)
        merged = oracle.merge_updates_v1(ups, mode=1)
        half = oracle.merge_updates_v1(ups[: len(ups) // 2], mode=1)
        sv = oracle.encode_state_vector_from_update_v1(half)
        diff = oracle.diff_updates_v1(merged, sv)
        rows.append({"merged": merged.hex(), "half": half.hex(), "diff": diff.hex(), "end": end})
        fx[name] = {"updates": len(ups), "update_bytes": int(b.data.size), "merged_len": len(merged),
                    "merged_sha256": sha(merged), "half_sha256": sha(half), "sv_half_sha256": sha(sv),
                    "diff_sha256": sha(diff), "end_len": len(end)}
        print(name, fx[name]["updates"], len(merged), flush=True)
    tmp = "/tmp/ymerge_traces_check.json"
    with open(tmp, "w") as f:
        json.dump(rows, f)
    js = os.path.join(os.path.dirname(os.path.abspath(__file__)), "check_traces.js")
    res = json.loads(subprocess.check_output(["node", js, tmp]))
    for name, r in zip(workloads.TRACES, res):
        fx[name].update(r)
    out = {"traces": "assets/editing-traces/sequential_traces/*.json.gz (copied to tests/golden/)",
           "check": "Yjs applyUpdate(oracle merge) text == endContent; Yjs applyUpdate(half merge) then "
                    "applyUpdate(oracle diff(merge, sv(half))) text == endContent",
           "results": fx}
    with open(os.path.join(ROOT, "tests", "golden", "traces_yjs_check.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
