"""Diagnostic: k_plan_wave windows / stitch rounds / hand-overs on C5-shaped documents
(YMERGE_STAMPS=1 stamps, marker 0xD1FE; never used for timed numbers)."""
import ctypes
import os
import sys

os.environ["YMERGE_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
import numpy as np  # noqa: E402
import workloads  # noqa: E402
import ymerge  # noqa: E402


def main(n=2000):
    e = ymerge.Engine(0)
    b = workloads.text_docs(n, 1000)
    out, off, st = e.merge_host(b.data, b.upd_off, b.doc_upd)
    sv, sv_off, _ = e.state_vector_host(out, off)
    rsv, rsv_off = workloads.remote_svs(sv, sv_off)
    for name, fn in (("diff", lambda: e.diff_host(out, off, rsv, rsv_off)), ("sv", lambda: e.state_vector_host(out, off))):
        fn()
        L = ymerge.lib()
        L.ymerge_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        s = np.zeros((n, 16), np.uint64)
        assert L.ymerge_debug_stamps(e._ctx, n, s.ctypes.data) == 0
        ok = s[:, 7] == 0xD1FE
        print(f"{name}: stamped {ok.sum()}/{n}, windows/doc {s[ok, 0].mean():.2f}, stitch rounds/doc "
              f"{s[ok, 1].mean():.2f} (max {s[ok, 1].max()}), handed over {int(s[ok, 2].sum())}, "
              f"bytes/doc {s[ok, 5].mean():.0f}")
    e.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2000)
