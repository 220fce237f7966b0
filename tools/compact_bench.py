"""Store-based compaction timing (ycompact_updates_v1_batch_device) on a resident batch, with
the CPU oracle on a bounded sample beside it.

  python tools/compact_bench.py [c2|c3|traces] [n_docs] [steps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "y-crdt_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import oracle  # noqa: E402
import workloads  # noqa: E402
import ymerge  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    if kind == "c2":
        b = workloads.text_docs(n, 1000)
    elif kind == "c3":
        b = workloads.zipf_docs(n)
    else:
        b, _ = workloads.trace_updates("automerge-paper")
    dev = torch.device("cuda", 0)
    eng = ymerge.Engine(0)
    t_b = torch.from_numpy(ymerge.padded(b.data)).to(dev)
    t_u = torch.from_numpy(np.ascontiguousarray(b.upd_off, np.uint64).view(np.int64)).to(dev)
    t_d = torch.from_numpy(np.ascontiguousarray(b.doc_upd, np.uint64).view(np.int64)).to(dev)
    torch.cuda.synchronize()
    args = (t_b.data_ptr(), b.n_bytes, t_u.data_ptr(), b.n_updates, t_d.data_ptr(), b.n_docs)
    r = eng.compact_device(*args)  # warm-up (scratch allocation)
    ts = []
    for _ in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = eng.compact_device(*args)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    st = eng.stats()
    out, off, status = r.to_host()
    ms = 1e3 * min(ts)
    print(f"{kind}: {b.n_docs} docs, {b.n_updates} updates, {b.n_bytes / 1e6:.1f} MB -> {len(out) / 1e6:.1f} MB; "
          f"device {ms:.2f} ms ({b.n_bytes / ms / 1e6:.2f} GB/s, {b.n_docs / ms * 1e3:.0f} docs/s); "
          f"k_compact {st['ms_exact']:.2f} ms, counts+scan {st['ms_decode']:.2f} ms; "
          f"status {np.bincount(status, minlength=22)[[0, 21]].tolist()}", flush=True)
    # CPU oracle on a sample of documents (8 threads)
    k = min(b.n_docs, 1000)
    s = b.prefix(k) if hasattr(b, "prefix") else b
    t0 = time.perf_counter()
    arena, aoff, ost = oracle.compact_batch(s.data, s.upd_off, s.doc_upd, threads=8)
    dt = time.perf_counter() - t0
    print(f"oracle (8 threads) on {k} docs: {dt * 1e3:.1f} ms ({s.n_bytes / dt / 1e9:.3f} GB/s, {k / dt:.0f} docs/s)")
    ok = all(out[int(off[d]):int(off[d + 1])].tobytes() == arena[int(aoff[d]):int(aoff[d + 1])]
             for d in range(k) if status[d] == 0)
    print("sample parity", ok)


if __name__ == "__main__":
    main()
