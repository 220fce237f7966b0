"""Diagnostic: per-step k_lean time on the C3 batch (variance check) and the per-document
cycle distribution of its largest documents (YMERGE_STAMPS build)."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import workloads  # noqa: E402
import ymerge  # noqa: E402

b = workloads.zipf_docs(1_000_000, seed=0x5EED)
dev = torch.device("cuda", 0)
tb = torch.from_numpy(ymerge.padded(b.data)).to(dev)
tu = torch.from_numpy(b.upd_off.view(np.int64)).to(dev)
td = torch.from_numpy(b.doc_upd.view(np.int64)).to(dev)
e = ymerge.Engine(0)
for i in range(8):
    torch.cuda.synchronize()
    t = time.perf_counter()
    e.merge_device(tb.data_ptr(), b.n_bytes, tu.data_ptr(), len(b.upd_off) - 1, td.data_ptr(), b.n_docs)
    w = (time.perf_counter() - t) * 1e3
    st = e.stats()
    print(f"step {i}: wall {w:.2f} ms, k_lean {st['ms_lean']:.2f} ms, lean docs {st['docs_lean']}", flush=True)
U = np.diff(b.doc_upd.astype(np.int64))
print("docs > 1280 updates:", int((U > 1280).sum()), "max U", int(U.max()), "bytes in big docs",
      int(sum(b.upd_off[b.doc_upd[1:]][U > 1280] - b.upd_off[b.doc_upd[:-1]][U > 1280])))
