"""Diagnostic: k_lean hand-over reasons (env YMERGE_LEAN_DEBUG) for test_lean_big_documents' docs."""
import os
import sys
os.environ["YMERGE_LEAN_DEBUG"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "oracle", "y-crdt_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
import ymerge  # noqa: E402
from test_gpu_lean import item, text_log, upd  # noqa: E402
from test_gpu_parity import batch_of  # noqa: E402

rng = np.random.default_rng(0xB1C)
docs = []
for n in (1281, 2000, 5000, 12000):
    cl = [int(x) for x in rng.integers(0, 2 ** 32, int(rng.integers(1, 6)))]
    docs.append(text_log(rng, cl, n))
docs.append(text_log(rng, [7], 3000, del_frac=0.6))
ups, clock = [], 0
for i in range(700):
    t = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, 90))
    ups.append(upd(1, clock, item(t, origin=(1, clock - 1) if clock else None)))
    clock += len(t)
docs.append(ups)
ups = [upd(1, 0, item("x" * 500))]
for i in range(400):
    ups.append(upd(ds=[(1, [(i, 1), (i + 100, 1)])]))
docs.append(ups)
docs.append([upd(3, 0, item("a" * 600)), upd(3, 600, item("b" * 300))] +
            [upd(ds=[(3, [(2 * (i % 450), 1)])]) for i in range(1500)])
docs = docs[5:]
e = ymerge.Engine(0)
for i, d in enumerate(docs):
    b = batch_of([d])
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    print(i, len(d), e.stats()["docs_lean"], flush=True)
