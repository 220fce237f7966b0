"""Diagnostic: device time of merge / SV / diff over b4-update.bin (the reference's giant update)."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import corpus  # noqa: E402
import ymerge  # noqa: E402

u = corpus.b4_update()
e = ymerge.Engine(0)
data = np.frombuffer(u, np.uint8)
off = np.array([0, len(u)], np.uint64)
doc = np.array([0, 1], np.uint64)
for it in range(3):
    t0 = time.perf_counter()
    e.merge_host(data, off, doc)
    t1 = time.perf_counter()
    print(f"merge b4: {1e3 * (t1 - t0):.2f} ms host-timed, stats {e.stats()}")

# state vector and diff of the same update (remote state vector: half the client's clock)
def _var(x):
    out = bytearray()
    while True:
        b7 = x & 0x7F
        x >>= 7
        out.append(b7 | (0x80 if x else 0))
        if not x:
            return bytes(out)


sv = b"\x01" + _var(992_525_821) + _var(182_315 // 2)
for it in range(2):
    t0 = time.perf_counter()
    e.state_vector_host(data, off)
    t1 = time.perf_counter()
    e.diff_host(data, off, np.frombuffer(sv, np.uint8), np.array([0, len(sv)], np.uint64))
    t2 = time.perf_counter()
    print(f"b4 state vector {1e3 * (t1 - t0):.2f} ms, diff {1e3 * (t2 - t1):.2f} ms (host-timed)")
