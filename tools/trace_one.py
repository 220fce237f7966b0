"""Diagnostic: merge one editing trace as a single document (kernel times under rocprofv3)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "y-crdt_amd"))
import workloads  # noqa: E402
import ymerge  # noqa: E402

b, _ = workloads.trace_updates(sys.argv[1])
e = ymerge.Engine(0)
for _ in range(3):
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    st = e.stats()
    print(sys.argv[1], {k: round(v, 3) for k, v in st.items() if k.startswith("ms_") and v}, st["docs_giant"], flush=True)
