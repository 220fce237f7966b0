import os, sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'y-crdt_amd'); sys.path.insert(0, 'oracle')
os.environ["YMERGE_LEAN_DEBUG"] = "1"
import numpy as np
import test_gpu_lean as T
from test_gpu_parity import batch_of
import ymerge
e = ymerge.Engine(0)
rng = np.random.default_rng(0x1EA4)
docs = [
    [T.upd(7, 0, T.item("ab")), T.upd(7, 2, T.item("c", origin=(7, 1))), T.upd(3, 0, T.item("xyz"))],
    [T.upd(5, 0, T.gc(3)), T.upd(5, 3, T.gc(2)), T.upd(5, 5, T.item("q"))],
    [T.upd(ds=[(4, [(0, 3)])]), T.upd(ds=[(4, [(3, 2)]), (8, [(10, 1)])])],
]
for n in (1, 5, 63, 64, 65, 130, 700, 1000):
    docs.append(T.text_log(rng, [int(x) for x in rng.integers(0, 2 ** 32, int(rng.integers(1, 6)))], n))
for i, d in enumerate(docs):
    b = batch_of([d])
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    print(i, len(d), e.stats()["docs_lean"], flush=True)
import workloads
b = workloads.text_docs(200, 1000)
e.merge_host(b.data, b.upd_off, b.doc_upd); print("c2", e.stats()["docs_lean"], flush=True)
b = workloads.zipf_docs(5000)
e.merge_host(b.data, b.upd_off, b.doc_upd); print("c3", e.stats()["docs_lean"], flush=True)
