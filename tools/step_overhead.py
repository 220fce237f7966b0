"""Diagnostic: the fixed host cost of one merge_device call (a 1-document batch, the kernels
trivially short) next to the C2 step and its k_lean time."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import workloads  # noqa: E402
import ymerge  # noqa: E402

dev = torch.device("cuda:0")
e = ymerge.Engine(0)
for name, b, n in (("tiny", workloads.text_docs(1, 10, seed=3), 2000), ("C2", workloads.text_docs(10000, 1000), 50)):
    t_b = torch.from_numpy(ymerge.padded(b.data)).to(dev)
    t_u = torch.from_numpy(b.upd_off.view(np.int64)).to(dev)
    t_d = torch.from_numpy(b.doc_upd.view(np.int64)).to(dev)
    args = (t_b.data_ptr(), b.n_bytes, t_u.data_ptr(), b.n_updates, t_d.data_ptr(), b.n_docs)
    for _ in range(5):
        e.merge_device(*args)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(n):
        e.merge_device(*args)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / n
    st = e.stats()
    print(f"{name}: {dt * 1e6:.1f} us per call, ms_lean {st['ms_lean']:.3f} ms_total {st['ms_total']:.3f}", flush=True)
