"""Diagnostic: C4 merge timings over repeated calls (merge_host and merge_device)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
import torch  # noqa: E402
import workloads  # noqa: E402
import ymerge  # noqa: E402

b = workloads.delete_heavy_docs(2000, 5000)
e = ymerge.Engine(0)
for k in range(3):
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    s = e.stats()
    print("host", k, round(s["ms_decode"], 3), round(s["ms_big"], 3), s["docs_big"], s["docs_exact"])
dev = torch.device("cuda:0")
t_b = torch.from_numpy(ymerge.padded(b.data)).to(dev)
t_u = torch.from_numpy(b.upd_off.view("int64")).to(dev)
t_d = torch.from_numpy(b.doc_upd.view("int64")).to(dev)
for k in range(3):
    e.merge_device(t_b.data_ptr(), b.n_bytes, t_u.data_ptr(), b.n_updates, t_d.data_ptr(), b.n_docs)
    s = e.stats()
    print("dev", k, round(s["ms_decode"], 3), round(s["ms_big"], 3), s["docs_big"], s["docs_exact"])
