"""Diagnostic: merge_updates_v2 stage times (v2 -> v1x decode, merge, v1x -> v2 encode) on C2-shaped
documents (workloads.text_docs), inputs converted on the device first."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "y-crdt_amd"))
import numpy as np  # noqa: E402
import workloads  # noqa: E402
import ymerge  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
b = workloads.text_docs(n, 1000)
e = ymerge.Engine(0)
v2b, v2off, st = e.convert_v1_to_v2_host(b.data, b.upd_off)
assert not st.any()
for it in range(3):
    out, off, st = e.merge_host(v2b[:int(v2off[-1])], v2off, b.doc_upd, version=2)
    s = e.stats()
    print(f"v2 merge of {n} docs: decode {s['ms_v2_decode']:.2f} merge {s['ms_v2_merge']:.2f} "
          f"encode {s['ms_v2_encode']:.2f} ms, status errors {int((st != 0).sum())}")
