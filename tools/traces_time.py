"""Diagnostic: device stage times of merge_updates_v1 over the five editing traces (one document each)."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'y-crdt_amd'))
import workloads, ymerge
b = workloads.traces_batch()
e = ymerge.Engine(0)
for it in range(3):
    t = time.perf_counter(); e.merge_host(b.data, b.upd_off, b.doc_upd); t1 = time.perf_counter()
    st = e.stats()
    print(f"traces ({b.n_docs} docs, {b.n_updates} updates) merge {1e3*(t1-t):.2f} ms host, decode {st['ms_decode']:.2f} "
          f"fast {st['ms_fast']:.2f} big {st['ms_big']:.2f} exact {st['ms_exact']:.2f} lean {st['ms_lean']:.2f} "
          f"total {st['ms_total']:.2f} giant {st['docs_giant']} big {st['docs_big']}")
