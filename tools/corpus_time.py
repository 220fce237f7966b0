"""Diagnostic: device stage times of merge_updates_v1 over the reference corpus (small-test-dataset.bin,
5,320 documents), optionally tiled to N documents (bench.py --workload corpus uses 106,400)."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'y-crdt_amd'))
import workloads, ymerge
b = workloads.dataset_docs()
if len(sys.argv) > 1:
    b = workloads.tile(b, int(sys.argv[1]))
e = ymerge.Engine(0)
for it in range(3):
    t = time.perf_counter(); e.merge_host(b.data, b.upd_off, b.doc_upd); t1 = time.perf_counter()
    st = e.stats()
    print(f"corpus ({b.n_docs} docs) merge {1e3*(t1-t):.2f} ms host, decode {st['ms_decode']:.2f} fast {st['ms_fast']:.2f} "
          f"big {st['ms_big']:.2f} exact {st['ms_exact']:.2f} lean {st['ms_lean']:.2f} total {st['ms_total']:.2f}")
