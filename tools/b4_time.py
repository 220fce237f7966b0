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
