"""Diagnostic: per-phase cycle shares of k_fast_merge (s_memtime stamps, separate
instantiation enabled by YMERGE_STAMPS=1; never used for timed numbers)."""
import ctypes
import os
import sys

os.environ["YMERGE_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
import numpy as np  # noqa: E402
import workloads  # noqa: E402
import ymerge  # noqa: E402

NAMES = ["decode", "-", "sort", "classify", "sizes", "write", "ds_clients", "ds_order", "ds_rsort", "ds_union",
         "ds_write"]


BIG_NAMES = ["gather", "sort", "classify", "write", "deleteset"]


def main_big(n, kind="c3"):
    """Tiled-kernel documents (k_big_merge, marker 0xB16 in slot 7) of a C3-style (or C4) batch."""
    if kind == "traces":
        b = workloads.traces_batch()
        n = b.n_docs
    else:
        b = workloads.zipf_docs(n, seed=0x5EED) if kind == "c3" else workloads.delete_heavy_docs(n)
    e = ymerge.Engine(0)
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    L = ymerge.lib()
    L.ymerge_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    st = np.zeros((n, 16), np.uint64)
    assert L.ymerge_debug_stamps(e._ctx, n, st.ctypes.data) == 0
    ok = (st[:, 7] == 0xB16) & (st[:, 5] > 0)
    U = np.diff(b.doc_upd.astype(np.int64))[ok]
    d = np.diff(st[ok][:, :6].astype(np.int64), axis=1)
    tot = d.sum(axis=1)
    print(f"tiled docs: {ok.sum()}, updates/doc mean {U.mean():.0f}, cycles/doc mean {tot.mean():.0f}, "
          f"cycles/update {(tot / U).mean():.0f}")
    s = st[ok].astype(np.int64)
    om = s[:, 8] > 0
    if om.any():
        print(f"  classify: {om.sum()} docs in overlap mode: pass 0 {(s[om, 8] - s[om, 2]).mean():.0f}, "
              f"run order {(s[om, 9] - s[om, 8]).mean():.0f}, pass 1 {(s[om, 3] - s[om, 9]).mean():.0f}")
        print(f"  run order: runs {(s[om, 6] - s[om, 8]).mean():.0f}, predecessors {(s[om, 13] - s[om, 6]).mean():.0f}, "
              f"sort {(s[om, 14] - s[om, 13]).mean():.0f}, tie rounds {(s[om, 15] - s[om, 14]).mean():.0f}, "
              f"GC ties + positions {(s[om, 9] - s[om, 15]).mean():.0f}")
    print(f"  deleteset: table+order {(s[:, 10] - s[:, 4]).mean():.0f}, range sort {(s[:, 11] - s[:, 10]).mean():.0f}, "
          f"union {(s[:, 12] - s[:, 11]).mean():.0f}, write {(s[:, 5] - s[:, 12]).mean():.0f}")
    for i, nm in enumerate(BIG_NAMES):
        print(f"  {nm:10s} {d[:, i].mean():10.0f} cycles  {100 * d[:, i].mean() / tot.mean():5.1f}%")
    for lo, hi in ((0, 2000), (2000, 4000), (4000, 10001)):
        sel = (U > lo) & (U <= hi)
        if sel.any():
            print(f"  U in ({lo},{hi}]: {sel.sum()} docs, cycles/doc {tot[sel].mean():.0f}, "
                  + ", ".join(f"{nm} {d[sel, i].mean():.0f}" for i, nm in enumerate(BIG_NAMES)))


def main_c1():
    """The automerge-paper trace as one document (C1): tiled-kernel phase split."""
    b, _ = workloads.trace_updates("automerge-paper")
    e = ymerge.Engine(0)
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    L = ymerge.lib()
    L.ymerge_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    st = np.zeros((1, 16), np.uint64)
    assert L.ymerge_debug_stamps(e._ctx, 1, st.ctypes.data) == 0
    d = np.diff(st[0, :6].astype(np.int64))
    print("marker", hex(int(st[0, 7])), "stats", e.stats())
    for i, nm in enumerate(BIG_NAMES):
        print(f"  {nm:10s} {d[i]:10d} cycles ({d[i] / 100e3:.3f} ms at 100 MHz)  {100 * d[i] / d.sum():5.1f}%")


def main_compact(n, lpw):
    """k_compact (store-based compaction) of C2 documents: per-document phase cycle sums."""
    os.environ["YMERGE_COMPACT_LPW"] = str(lpw)
    b = workloads.text_docs(n, 1000)
    e = ymerge.Engine(0)
    e.compact_host(b.data, b.upd_off, b.doc_upd)
    L = ymerge.lib()
    L.ymerge_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    st = np.zeros((n, 16), np.uint64)
    assert L.ymerge_debug_stamps(e._ctx, n, st.ctypes.data) == 0
    print(f"compact docs {n}, lpw {lpw}: {e.stats()['ms_exact']:.2f} ms k_compact")
    tot = st[:, :5].sum(axis=1).astype(np.float64)
    upd = np.maximum(st[:, 5].astype(np.float64), 1)
    print(f"  cycles/doc {tot.mean():.0f}, cycles/update {(tot / upd).mean():.0f}")
    for i, nm in enumerate(["decode", "integrate", "apply_delete", "commit", "encode"]):
        v = st[:, i].astype(np.float64)
        print(f"  {nm:12s} {v.mean():12.0f} cycles/doc {(v / upd).mean():8.0f} /update {100 * v.mean() / tot.mean():5.1f}%")


def main_c5(n):
    """k_plan_ring (diff planner) on C5-style documents (C2 merge outputs vs remote SVs)."""
    b = workloads.text_docs(n, 1000)
    e = ymerge.Engine(0)
    out, off, st = e.merge_host(b.data, b.upd_off, b.doc_upd)
    db = workloads.compacted_docs(out, off, sv_fn=lambda dd, oo: e.state_vector_host(dd, oo))
    e.diff_host(db.data, db.upd_off, db.sv, db.sv_off)
    L = ymerge.lib()
    L.ymerge_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    stt = np.zeros((n, 16), np.uint64)
    assert L.ymerge_debug_stamps(e._ctx, n, stt.ctypes.data) == 0
    ok = stt[:, 7] == 0xD1FF
    s = stt[ok].astype(np.float64)
    print(f"k_plan_ring docs {ok.sum()} of {n}, stats {e.stats()}")
    print(f"  bytes/doc {s[:, 5].mean():.0f}; wave cycles: refill {s[:, 0].mean():.0f} ({s[:, 3].mean():.0f} rounds), "
          f"steps {s[:, 1].mean():.0f} ({s[:, 4].mean():.0f} iterations), finish {s[:, 2].mean():.0f}")
    print(f"  cycles per step iteration {(s[:, 1] / np.maximum(s[:, 4], 1)).mean():.0f}, "
          f"per refill {(s[:, 0] / np.maximum(s[:, 3], 1)).mean():.0f}")


def main_zipf(n):
    """Fast-path documents of a C3-style batch, phase cycles by update count."""
    b = workloads.zipf_docs(n, seed=0x5EED)
    e = ymerge.Engine(0)
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    L = ymerge.lib()
    L.ymerge_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    st = np.zeros((n, 16), np.uint64)
    assert L.ymerge_debug_stamps(e._ctx, n, st.ctypes.data) == 0
    ok = (st[:, 11] > 0) & (st[:, 7] != 0xB16)
    U = np.diff(b.doc_upd.astype(np.int64))[ok]
    d = np.diff(st[ok][:, :12].astype(np.int64), axis=1)
    tot = d.sum(axis=1)
    print(f"fast docs {ok.sum()}: cycles/doc mean {tot.mean():.0f}")
    for lo, hi in ((0, 4), (4, 16), (16, 64), (64, 256), (256, 1300)):
        sel = (U > lo) & (U <= hi)
        if sel.any():
            print(f"  U in ({lo},{hi}]: {sel.sum()} docs, cycles/doc {tot[sel].mean():.0f}: "
                  + ", ".join(f"{nm} {d[sel, i].mean():.0f}" for i, nm in enumerate(NAMES) if nm != "-"))


def main_corpus():
    """The reference corpus (small-test-dataset.bin, 5,320 documents): fast-path phase cycles,
    records still walked over HBM (REC_SLOW) and re-walked (fill), and the slowest documents."""
    b = workloads.dataset_docs()
    e = ymerge.Engine(0)
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    L = ymerge.lib()
    L.ymerge_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    n = b.n_docs
    st = np.zeros((n, 16), np.uint64)
    assert L.ymerge_debug_stamps(e._ctx, n, st.ctypes.data) == 0
    print("stats", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in e.stats().items()})
    fast = (st[:, 11] > 0) & (st[:, 7] != 0xB16)
    big = st[:, 7] == 0xB16
    U = np.diff(b.doc_upd.astype(np.int64))
    nbytes = np.diff(b.upd_off[b.doc_upd.astype(np.int64)].astype(np.int64))
    d = np.diff(st[fast][:, :12].astype(np.int64), axis=1)
    tot = d.sum(axis=1)
    print(f"fast docs {fast.sum()}, big docs {big.sum()}; fast cycles/doc mean {tot.mean():.0f}, max {tot.max()}")
    print("  phases: " + ", ".join(f"{nm} {d[:, i].mean():.0f}" for i, nm in enumerate(NAMES) if nm != "-"))
    print(f"  records: slow {st[fast, 12].sum()}, complex {st[fast, 13].sum()}, fill walks {st[fast, 14].sum()}, "
          f"overflow words {st[fast, 15].sum()}")
    idx = np.nonzero(fast)[0][np.argsort(-tot)[:8]]
    for q in idx:
        dd = np.diff(st[q, :12].astype(np.int64))
        print(f"  doc {q}: U {U[q]} bytes {nbytes[q]} slow {st[q, 12]} cx {st[q, 13]}: "
              + ", ".join(f"{nm} {dd[i]}" for i, nm in enumerate(NAMES) if nm != "-"))
    if big.any():
        db = np.diff(st[big][:, :6].astype(np.int64), axis=1)
        print(f"big docs: U {U[big].tolist()[:10]} bytes {nbytes[big].tolist()[:10]}")
        print("  cycles/doc " + ", ".join(f"{nm} {db[:, i].mean():.0f}" for i, nm in enumerate(BIG_NAMES)))


LEAN_NAMES = ["init", "decode", "layout", "copy", "ds_union", "ds_write"]
LEAN_SUB = ["stage+prefetch", "walk", "blocks", "deleteset"]


def main_lean(kind, n):
    """k_lean documents (marker 0x1EA4 in slot 15): phase cycles, decode sub-phases per round."""
    b = workloads.text_docs(n, 1000) if kind == "c2" else workloads.zipf_docs(n, seed=0x5EED)
    e = ymerge.Engine(0)
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    L = ymerge.lib()
    L.ymerge_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    st = np.zeros((n, 16), np.uint64)
    assert L.ymerge_debug_stamps(e._ctx, n, st.ctypes.data) == 0
    ok = st[:, 15] == 0x1EA4
    U = np.diff(b.doc_upd.astype(np.int64))[ok]
    d = np.diff(st[ok][:, :7].astype(np.int64), axis=1)
    tot = d.sum(axis=1)
    rounds = st[ok][:, 12].astype(np.float64)
    print(f"lean docs {ok.sum()} of {n}: cycles/doc mean {tot.mean():.0f}, rounds/doc {rounds.mean():.1f}, "
          f"updates/doc {U.mean():.0f}")
    for i, nm in enumerate(LEAN_NAMES):
        print(f"  {nm:10s} {d[:, i].mean():10.0f} cycles  {100 * d[:, i].mean() / tot.mean():5.1f}%")
    for i, nm in enumerate(LEAN_SUB):
        v = st[ok][:, 8 + i].astype(np.float64)
        print(f"  decode/{nm:16s} {v.mean():10.0f} cycles/doc  {(v / np.maximum(rounds, 1)).mean():8.0f} per round")
    dsp, npass = st[ok][:, 13].astype(np.float64), st[ok][:, 14].astype(np.float64)
    print(f"  ds_union = DeleteSet batches: {dsp.mean():.0f} cycles/doc, {npass.mean():.1f} batches/doc, "
          f"{(dsp / np.maximum(npass, 1)).mean():.0f} cycles/batch")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "lean":
        return main_lean(sys.argv[2] if len(sys.argv) > 2 else "c2", int(sys.argv[3]) if len(sys.argv) > 3 else 10000)
    if len(sys.argv) > 1 and sys.argv[1] == "zipf":
        os.environ["YMERGE_TINY"] = "0"
        return main_zipf(int(sys.argv[2]) if len(sys.argv) > 2 else 20000)
    if len(sys.argv) > 1 and sys.argv[1] == "big":
        return main_big(int(sys.argv[2]) if len(sys.argv) > 2 else 20000)
    if len(sys.argv) > 1 and sys.argv[1] == "traces":
        return main_big(0, "traces")
    if len(sys.argv) > 1 and sys.argv[1] == "c4":
        return main_big(int(sys.argv[2]) if len(sys.argv) > 2 else 2000, "c4")
    if len(sys.argv) > 1 and sys.argv[1] == "c1":
        return main_c1()
    if len(sys.argv) > 1 and sys.argv[1] == "corpus":
        return main_corpus()
    if len(sys.argv) > 1 and sys.argv[1] == "c5":
        return main_c5(int(sys.argv[2]) if len(sys.argv) > 2 else 20000)
    if len(sys.argv) > 1 and sys.argv[1] == "compact":
        return main_compact(int(sys.argv[2]) if len(sys.argv) > 2 else 10000, int(sys.argv[3]) if len(sys.argv) > 3 else 16)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    threads = os.environ.get("YMERGE_FAST_THREADS", "256")
    b = workloads.text_docs(n, 1000)
    e = ymerge.Engine(0)
    e.merge_host(b.data, b.upd_off, b.doc_upd)
    L = ymerge.lib()
    L.ymerge_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    st = np.zeros((n, 16), np.uint64)
    assert L.ymerge_debug_stamps(e._ctx, n, st.ctypes.data) == 0
    ok = st[:, 11] > 0
    d = np.diff(st[ok][:, :12].astype(np.int64), axis=1)
    tot = d.sum(axis=1).mean()
    print(f"threads/WG {threads}: {ok.sum()} fast docs, mean {tot:.0f} cycles per doc")
    print("  per doc: %.1f updates walked over HBM (outside the stage), %.1f multi-record updates" % (st[ok][:, 12].mean(), st[ok][:, 13].mean()))
    print("  per doc: %.1f multi-record updates re-walked over HBM" % st[ok][:, 14].mean())
    for i, nm in enumerate(NAMES):
        print(f"  {nm:10s} {d[:, i].mean():10.0f} cycles  {100 * d[:, i].mean() / tot:5.1f}%")


if __name__ == "__main__":
    main()
