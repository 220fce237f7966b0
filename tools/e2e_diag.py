"""Diagnostic: where the C-ABI host entry (ymerge_updates_v1_batch) spends its time on C2."""
import ctypes
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
import numpy as np  # noqa: E402
import workloads  # noqa: E402
import ymerge  # noqa: E402

b = workloads.text_docs(10000, 1000)
e = ymerge.Engine(0)
L = ymerge.lib()
for i in range(4):
    pres = ctypes.c_void_p()
    t0 = time.perf_counter()
    rc = L.ymerge_updates_v1_batch(e._ctx, b.data.ctypes.data, b.upd_off.ctypes.data, b.n_updates,
                                   b.doc_upd.ctypes.data, b.n_docs, ctypes.byref(pres))
    t1 = time.perf_counter()
    r = ymerge._BatchRes.from_address(pres.value)
    t2 = time.perf_counter()
    L.ymerge_batch_result_destroy(pres)
    t3 = time.perf_counter()
    print(f"call {1e3 * (t1 - t0):.1f} ms ({b.n_bytes / (t1 - t0) / 1e9:.1f} GB/s in), destroy {1e3 * (t3 - t2):.1f} ms,"
          f" out {r.out_bytes}", flush=True)
import torch  # noqa: E402
hb = torch.from_numpy(b.data).pin_memory()
for i in range(3):
    pres = ctypes.c_void_p()
    t0 = time.perf_counter()
    rc = L.ymerge_updates_v1_batch(e._ctx, hb.data_ptr(), b.upd_off.ctypes.data, b.n_updates,
                                   b.doc_upd.ctypes.data, b.n_docs, ctypes.byref(pres))
    t1 = time.perf_counter()
    L.ymerge_batch_result_destroy(pres)
    print(f"pinned input: call {1e3 * (t1 - t0):.1f} ms ({b.n_bytes / (t1 - t0) / 1e9:.1f} GB/s in)", flush=True)
st = e.stats()
print({k: round(v, 3) if isinstance(v, float) else v for k, v in st.items()})
