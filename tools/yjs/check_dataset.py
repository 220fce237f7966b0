"""TEST TOOLING ONLY (this container): pins the oracle on the reference's real corpus.

For every document of tests/golden/small-test-dataset.bin (the corpus of
yrs/src/tests/compatibility_tests.rs:427-476) the CPU oracle merges the document's
updates (merge_updates_v1, literal and fast modes must agree), then the offline Yjs
bundle applies the merged update to a fresh Y.Doc and its "text" / "map" / "array"
values are compared with the values the corpus records.  Writes the summary fixture
tests/golden/small_dataset_yjs_check.json (per-document status + sha256 of the merge).

    python tools/yjs/check_dataset.py
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import corpus  # noqa: E402
import oracle  # noqa: E402


def main():
    docs = corpus.small_dataset()
    merged, rows = [], []
    for k, (ups, text, m, a) in enumerate(docs):
        out = oracle.merge_updates_v1(ups, mode=1)
        assert oracle.merge_updates_v1(ups, mode=0) == out, k
        merged.append(out)
        rows.append({"merged": out.hex(), "text": text, "map": m, "array": a})
    tmp = "/tmp/ymerge_dataset_check.json"
    with open(tmp, "w") as f:
        json.dump(rows, f)
    js = os.path.join(os.path.dirname(os.path.abspath(__file__)), "check_dataset.js")
    res = json.loads(subprocess.check_output(["node", js, tmp]))
    fixture = {
        "corpus": "assets/bench-input/small-test-dataset.bin (copied as tests/golden/small-test-dataset.bin)",
        "check": "oracle merge_updates_v1 of each document applied by the offline Yjs bundle; Y.Text/Y.Map/"
                 "Y.Array values compared with the values the corpus records",
        "docs": len(docs),
        "text_equal": res["text"], "map_equal": res["map"], "array_equal": res["array"],
        "failures": res["failures"][:20],
        "merge_sha256": [hashlib.sha256(o).hexdigest()[:16] for o in merged],
    }
    with open(os.path.join(ROOT, "tests", "golden", "small_dataset_yjs_check.json"), "w") as f:
        json.dump(fixture, f, indent=0)
    print({k: v for k, v in fixture.items() if k != "merge_sha256"})


if __name__ == "__main__":
    main()
