"""Benchmark: batched merge_updates_v1 / diff_updates_v1 on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c1|c2|c3|c4|c5] [--docs D] [--ops O]

Workloads (BASELINE.json configs; inputs resident in HBM before the timed region):
  c2 (default, configs[1])  per GPU D=10,000 synthetic YText docs x O=1,000 single-op v1 updates
                            (1-4 synced clients, 80/20 insert/delete); weak scaling
  c1 (configs[0])           the automerge-paper trace as 259,778 per-op updates, one document
  c3 (configs[2])           1,000,000 docs with Zipf(1.5) update counts on [1, 1e4], doc-hash
                            sharded over the ranks (total work fixed: strong scaling)
  c4 (configs[3])           2,000 delete-heavy docs x 5,000 updates (GC'd snapshot + per-op log)
  c5 (configs[4])           diff_updates_v1 of 100,000 compacted docs (C2 merge outputs) against
                            per-document remote state vectors (sync-step-2 serving); weak scaling
  corpus                    the reference's real inputs: small-test-dataset.bin's 5,320 documents tiled
                            to D=106,400 per GPU, plus the five editing traces batched (a second block)
One step = one full batched call over the GPU's shard.  For N > 1 (torch.distributed.run,
one rank per GPU) documents are sharded by splitmix64(doc_id) % N with no data-path
collective; RCCL carries the barrier, the max-over-ranks time and a per-shard stats gather.

Prints ONE JSON line (rank 0).  `value` = input GB/s over all ranks; docs/s, the roofline
of the device pipeline (HIP events on the engine's stream), an end-to-end number (H2D +
pipeline + pack + D2H) and the CPU baseline (the oracle, literal yrs algorithm, bounded
sample, rank 0, N=1) ride along.
"""
import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "input GB/s + docs compacted/sec, batched merge_updates_v1 @ 1/2/4/8 GPUs"
METRIC_DIFF = "input GB/s + docs served/sec, batched diff_updates_v1 (sync-step-2) @ 1/2/4/8 GPUs"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); > 1 without WORLD_SIZE starts them via torch.distributed.run")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "corpus"])
    ap.add_argument("--docs", type=int, default=None, help="documents (per GPU for c2/c4/c5, total for c3)")
    ap.add_argument("--ops", type=int, default=None, help="updates per document (c2/c4/c5)")
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="target wall time of one CPU-baseline run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-compact", action="store_true", help="skip the store-based compaction line (c2)")
    ap.add_argument("--no-v2", action="store_true", help="skip the merge_updates_v2 line of the C2 documents (lib0_v2)")
    return ap.parse_args()


def pmc_traffic(workload):
    """HBM bytes per launch of the pipeline from a committed rocprofv3 PMC pass, if any."""
    p = os.path.join(ROOT, "profiles", f"pmc_traffic_{workload}.json")
    if os.path.exists(p):
        try:
            with open(p) as f:
                d = json.load(f)
            if d.get("workload", "c2") == workload:
                return d.get("traffic_bytes_per_launch")
        except Exception:
            return None
    return None


def host_cpu():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        share = min(share, int(env))  # the GPU box's CPU share for this job
    return model, os.cpu_count() or 1, max(1, share)


def timed_runs(fn, runs):
    fn()  # warm-up
    ts = []
    for _ in range(runs):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts)


# ------------------------------------------------------------------ workloads
def build_merge(a, rank, world):
    import dist
    import workloads
    w = a.workload
    if w == "c1":
        batch, _ = workloads.trace_updates()
        return batch, "C1: automerge-paper trace as 259,778 per-op v1 updates, one document, merge_updates_v1", \
            "replicas", {"docs": 1, "updates": batch.n_updates}
    if w == "c2":
        docs, ops = a.docs or 10_000, a.ops or 1_000
        ids = dist.shard(world * docs, rank, world) if world > 1 else np.arange(docs, dtype=np.uint64)
        batch = workloads.text_docs(len(ids), ops, ids=ids)
        return batch, f"C2: {docs} synthetic YText docs x {ops} single-op v1 updates per GPU, batched " \
                      "merge_updates_v1", "weak", {"docs_per_gpu": docs, "updates_per_doc": ops}
    if w == "c3":
        docs = a.docs or 1_000_000
        ids = dist.shard(docs, rank, world) if world > 1 else np.arange(docs, dtype=np.uint64)
        batch = workloads.zipf_docs(docs, ids=ids) if world > 1 else workloads.zipf_docs(docs)
        return batch, f"C3: {docs} docs total, Zipf(1.5) update counts on [1, 1e4], doc-hash sharded, " \
                      "batched merge_updates_v1", "strong", {"docs_total": docs}
    if w == "c4":
        docs, ops = a.docs or 2_000, a.ops or 5_000
        batch = workloads.delete_heavy_docs(docs, ops)
        return batch, f"C4: {docs} delete-heavy docs x {ops} updates per GPU (70% deletes, GC'd snapshot + " \
                      "per-op log, withheld/duplicated updates)", "weak", {"docs_per_gpu": docs,
                                                                         "updates_per_doc": ops}
    if w == "corpus":
        docs = a.docs or 106_400
        batch = workloads.tile(workloads.dataset_docs(), docs)
        return batch, f"corpus: assets/bench-input/small-test-dataset.bin (5,320 real Yjs documents, " \
                      f"compatibility_tests.rs:437-476) tiled to {docs} docs per GPU, batched merge_updates_v1", \
            "weak", {"docs_per_gpu": docs}
    raise ValueError(w)


def run_traces(eng, dev):
    """The five assets/editing-traces sequential traces, one document each, in one batch."""
    import workloads
    import ymerge
    tb = workloads.traces_batch()
    t_b = torch.from_numpy(ymerge.padded(tb.data)).to(dev)
    t_u = torch.from_numpy(tb.upd_off.view(np.int64)).to(dev)
    t_d = torch.from_numpy(tb.doc_upd.view(np.int64)).to(dev)
    args = (t_b.data_ptr(), tb.n_bytes, t_u.data_ptr(), tb.n_updates, t_d.data_ptr(), tb.n_docs)
    eng.merge_device(*args)
    runs = []
    for _ in range(3):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        r = eng.merge_device(*args)
        torch.cuda.synchronize(dev)
        runs.append(time.perf_counter() - t)
    st = eng.stats()
    _, _, rst = r.to_host()
    dt = min(runs)
    return {"value": tb.n_bytes / dt / 1e9, "unit": "GB/s", "ms": dt * 1e3, "docs": tb.n_docs,
            "updates": tb.n_updates, "bytes_in": tb.n_bytes, "bytes_out": int(r.out_bytes),
            "error_docs": int((rst != 0).sum()), "paths": path_stats(st)}


def path_stats(st):
    """Documents and device ms per merge path (the routing table of DESIGN.md section 5)."""
    return {"docs_lean": int(st["docs_lean"]), "docs_fast": int(st["docs_fast"]), "docs_tiled": int(st["docs_big"]),
            "docs_grid": int(st["docs_giant"]), "docs_overlap": int(st["docs_overlap"]),
            "docs_exact": int(st["docs_exact"]), "docs_tiny": int(st["docs_tiny"]),
            "k_lean_ms": st["ms_lean"], "k_decode_ms": st["ms_decode"], "k_fast_merge_ms": st["ms_fast"],
            "tiled_grid_ms": st["ms_big"], "exact_ms": st["ms_exact"]}


def cpu_merge_baseline(batch, a):
    import oracle
    model, nproc, share = host_cpu()
    if batch.n_docs == 1:  # C1: one document, quadratic reference loop -> bounded prefix, 1 core
        n_pre = min(batch.n_updates, 60_000)
        data = batch.data[:int(batch.upd_off[n_pre])]
        uo, du = batch.upd_off[:n_pre + 1], np.array([0, n_pre], np.uint64)
        dt = timed_runs(lambda: oracle.merge_batch(data, uo, du, mode=0, threads=1), 3)
        return {"value": len(data) / dt / 1e9, "unit": "GB/s", "cores": 1, "kind": "port",
                "docs_per_s": 1 / dt, "cpu_model": model, "nproc": nproc,
                "sample": f"first {n_pre} updates of the trace ({len(data)} B) as one merge_updates_v1 call, "
                          f"oracle literal yrs loop (quadratic per-iteration decoder re-sort), 1 core, "
                          f"median of 3 after 1 warm-up: {dt:.3f} s"}
    # sample sized so one all-cores run takes ~cpu_seconds (assumes ~25 MB/s per core)
    per_doc = max(1, batch.n_bytes // max(1, batch.n_docs))
    n_all = int(min(batch.n_docs, max(16, a.cpu_seconds * 25e6 * share / per_doc)))
    n_one = int(min(batch.n_docs, max(4, a.cpu_seconds * 25e6 / per_doc)))
    s_all = batch.prefix(n_all)
    s_one = batch.prefix(n_one)
    t_all = timed_runs(lambda: oracle.merge_batch(s_all.data, s_all.upd_off, s_all.doc_upd, mode=0,
                                                  threads=share), 5)
    t_one = timed_runs(lambda: oracle.merge_batch(s_one.data, s_one.upd_off, s_one.doc_upd, mode=0, threads=1), 5)
    return {"value": s_all.n_bytes / t_all / 1e9, "unit": "GB/s", "cores": share, "kind": "port",
            "docs_per_s": n_all / t_all, "cpu_model": model, "nproc": nproc,
            "one_core": {"value": s_one.n_bytes / t_one / 1e9, "unit": "GB/s", "docs_per_s": n_one / t_one,
                         "sample_docs": n_one, "sample_bytes": s_one.n_bytes},
            "sample": f"first {n_all} docs of the same workload ({s_all.n_bytes} B), oracle literal yrs loop "
                      f"(per-iteration decoder re-sort, DS re-squash), {share} threads (the job's CPU share of "
                      f"{nproc} host CPUs), median of 5 after 1 warm-up: {t_all:.3f} s"}


def run_merge(a, rank, world, dev):
    import dist
    import ymerge
    batch, desc, scaling, cfg = build_merge(a, rank, world)
    t_b = torch.from_numpy(ymerge.padded(batch.data)).to(dev)  # 16-byte reads past the end
    t_u = torch.from_numpy(batch.upd_off.view(np.int64)).to(dev)
    t_d = torch.from_numpy(batch.doc_upd.view(np.int64)).to(dev)
    torch.cuda.synchronize(dev)
    eng = ymerge.Engine(dev.index)

    def step():
        return eng.merge_device(t_b.data_ptr(), batch.n_bytes, t_u.data_ptr(), batch.n_updates, t_d.data_ptr(),
                                batch.n_docs)

    # the timed steps run without the engine's stage-timing events (a server has no use for
    # them); the stage times come from the same number of untimed steps after the loop
    eng.set_stage_timing(False)
    for _ in range(a.warmup):
        step()
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_stage_timing(True)
    # per-stage HIP-event times from the same number of untimed steps (reading the stats is
    # not part of a step: the getter waits on the step's last event)
    kstats = []
    for _ in range(a.steps):
        res = step()
        kstats.append(eng.stats())

    out_bytes = res.out_bytes
    _, _, st = res.to_host()
    n_err = int((st != 0).sum())
    mean = lambda k: float(np.mean([s[k] for s in kstats]))  # noqa: E731
    ms_lean, ms_decode, ms_fast = mean("ms_lean"), mean("ms_decode"), mean("ms_fast")
    ms_big, ms_exact = mean("ms_big"), mean("ms_exact")
    ms_pipe = ms_lean + ms_decode + ms_fast + ms_big + ms_exact
    docs_lean = int(kstats[-1]["docs_lean"])
    docs_exact, docs_big = int(kstats[-1]["docs_exact"]), int(kstats[-1]["docs_big"])
    docs_tiny = int(kstats[-1]["docs_tiny"])

    e2e = e2e_abi = pcie = None
    if not a.no_e2e:  # end-to-end: pinned host arena -> H2D -> pipeline -> pack -> D2H
        h_b = torch.from_numpy(ymerge.padded(batch.data)).pin_memory()
        h_u = torch.from_numpy(batch.upd_off.view(np.int64)).pin_memory()
        h_d = torch.from_numpy(batch.doc_upd.view(np.int64)).pin_memory()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        g_b, g_u, g_d = (x.to(dev, non_blocking=True) for x in (h_b, h_u, h_d))
        torch.cuda.synchronize(dev)
        r = eng.merge_device(g_b.data_ptr(), batch.n_bytes, g_u.data_ptr(), batch.n_updates, g_d.data_ptr(),
                             batch.n_docs)
        r.to_host()
        e2e = time.perf_counter() - t
        del g_b, g_u, g_d
        # the server-facing C-ABI host entry (ymerge_updates_v1_batch): pageable host arrays
        # in, a library-owned host result out (pinned double-buffered staging inside)
        for _ in range(2):  # warm: the pinned result pool, the staging ring
            eng.host_batch("ymerge_updates_v1_batch", batch.data, batch.upd_off, batch.n_updates, batch.doc_upd,
                           copy=False)
        t = time.perf_counter()
        eng.host_batch("ymerge_updates_v1_batch", batch.data, batch.upd_off, batch.n_updates, batch.doc_upd,
                       copy=False)
        e2e_abi = time.perf_counter() - t
        # PCIe lower bound for the same bytes: pinned H2D of the input + D2H of the output
        h_o = torch.empty(out_bytes, dtype=torch.uint8).pin_memory()
        g = torch.empty(max(batch.n_bytes, out_bytes), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        g[:batch.n_bytes].copy_(h_b[:batch.n_bytes], non_blocking=True)
        torch.cuda.synchronize(dev)
        h_o.copy_(g[:out_bytes], non_blocking=True)
        torch.cuda.synchronize(dev)
        pcie = time.perf_counter() - t
        del g, h_o

    compact = v2 = traces = None
    if a.workload == "corpus" and rank == 0:
        try:
            traces = run_traces(eng, dev)
        except Exception as e:  # noqa: BLE001
            traces = {"error": repr(e)[:200]}
    if a.workload == "c2" and rank == 0:
        # secondary measurements after the timed region: a failure is reported in the line,
        # it never costs the headline
        if not a.no_compact:
            try:
                compact = run_compact(a, eng, batch, (t_b, t_u, t_d), dev, world)
            except Exception as e:  # noqa: BLE001
                compact = {"error": repr(e)[:200]}
        if not a.no_v2:
            try:
                v2 = run_v2(a, eng, batch, dev, world)
            except Exception as e:  # noqa: BLE001
                v2 = {"error": repr(e)[:200]}

    allst = dist.gather_stats([batch.n_docs, batch.n_bytes, out_bytes, n_err, elapsed, ms_pipe,
                               e2e or 0.0], device=dev)
    if rank != 0:
        return None
    t_max = float(allst[:, 4].max())
    docs_total = float(allst[:, 0].sum()) * a.steps
    bytes_in_total = float(allst[:, 1].sum()) * a.steps
    # roofline of the merge pipeline (k_lean -> k_decode + k_fast_merge for the documents it
    # hands over -> tiled / exact engines; together they are the path), algorithmic bytes =
    # input + output
    alg_bytes = batch.n_bytes + out_bytes
    achieved = alg_bytes / (ms_pipe * 1e-3) / 1e9
    cpu = None
    if not a.no_cpu_baseline and world == 1:
        cpu = cpu_merge_baseline(batch, a)
    line = {
        "metric": METRIC, "value": bytes_in_total / t_max / 1e9, "unit": "GB/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": t_max / a.steps * 1e3, "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u8", "data": "synthetic" if a.workload != "c1" else
        "automerge-paper editing trace (CC BY 4.0) replayed into per-op updates",
        "docs_per_s": docs_total / t_max,
        "config": dict({"workload": desc + ", inputs HBM-resident", "bytes_in_per_gpu": int(allst[0, 1]),
                        "bytes_out_per_gpu": int(allst[0, 2]), "updates_per_gpu": batch.n_updates,
                        "parallelism": f"doc-hash sharding x{world}", "error_docs": int(allst[:, 3].sum())},
                       **cfg),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(a.workload),
                     "kernel": "k_lean(+k_decode+k_fast_merge, k_big_merge, exact engine)", "kernel_ms": ms_pipe,
                     "k_lean_ms": ms_lean, "docs_lean": docs_lean,
                     "k_decode_ms": ms_decode, "k_fast_merge_ms": ms_fast, "big_path_ms": ms_big,
                     "exact_path_ms": ms_exact, "docs_big_path": docs_big, "docs_exact_path": docs_exact,
                     "docs_tiny_path": docs_tiny,
                     "alg_bytes_per_launch": alg_bytes,
                     "stage_note": f"kernel_ms and the stage times are HIP-event means over {a.steps} "
                                   "separate untimed steps run after the timed loop (same batch)"},
        "paths": path_stats(kstats[-1]),
        "end_to_end": None if e2e is None else {
            "value": float(allst[:, 1].sum()) / float(allst[:, 6].max()) / 1e9, "unit": "GB/s",
            "note": "pinned host arena -> H2D -> merge -> pack -> D2H (pageable numpy), one batch",
            "c_abi_host_entry": batch.n_bytes / e2e_abi / 1e9 if e2e_abi else None,
            "c_abi_note": "ymerge_updates_v1_batch from pageable host arrays to a host result, rank 0",
            "pcie_bound": batch.n_bytes / pcie / 1e9 if pcie else None,
            "pcie_note": "input GB/s if only the pinned H2D of the input and D2H of the output ran"},
        "cpu_baseline": cpu,
        "store_compaction": compact,
        "lib0_v2": v2,
    }
    if traces is not None:
        line["editing_traces"] = traces
    return line


def run_v2(a, eng, batch, dev, world):
    """merge_updates_v2 (yrs/src/alt.rs:35-48) of the same documents with every update in lib0
    v2 (converted on the device, yconvert_updates_v1_to_v2_batch_device), inputs resident;
    rank 0's shard, the oracle's v2 merge on a bounded sample beside it."""
    import ymerge
    v2b, v2off, st = eng.convert_v1_to_v2_host(batch.data, batch.upd_off)
    if st.any():
        return {"error": "conversion status", "docs": int((st != 0).sum())}
    n2 = int(v2off[-1])
    t_b = torch.from_numpy(ymerge.padded(v2b[:n2])).to(dev)
    t_u = torch.from_numpy(np.ascontiguousarray(v2off, np.uint64).view(np.int64)).to(dev)
    t_d = torch.from_numpy(batch.doc_upd.view(np.int64)).to(dev)
    torch.cuda.synchronize(dev)
    args = (t_b.data_ptr(), n2, t_u.data_ptr(), batch.n_updates, t_d.data_ptr(), batch.n_docs)
    eng.merge_device(*args, version=2)
    runs = []
    for _ in range(3):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        r = eng.merge_device(*args, version=2)
        torch.cuda.synchronize(dev)
        runs.append(time.perf_counter() - t)
    st_k = eng.stats()
    _, _, rst = r.to_host()
    dt = min(runs)
    cpu = None
    if not a.no_cpu_baseline and world == 1:
        import oracle
        k = min(batch.n_docs, 1000)
        u1 = int(batch.doc_upd[k])
        threads = min(16, os.cpu_count() or 1)
        t = time.perf_counter()
        oracle.merge_batch(v2b[:int(v2off[u1])], v2off[:u1 + 1], batch.doc_upd[:k + 1], mode=1, threads=threads,
                           version=2)
        ct = time.perf_counter() - t
        cpu = {"value": int(v2off[u1]) / ct / 1e9, "unit": "GB/s", "cores": threads, "kind": "port",
               "sample": f"oracle merge_updates_v2 (fast mode) on the first {k} documents"}
    alg = n2 + int(r.out_bytes)  # v2 in + v2 out (per launch)
    return {"value": n2 / dt / 1e9, "unit": "GB/s", "ms": dt * 1e3, "docs_per_s": batch.n_docs / dt,
            "v2_bytes_in": n2, "v2_bytes_out": int(r.out_bytes), "error_docs": int((rst != 0).sum()),
            "roofline": {"bound": "hbm", "achieved": alg / dt / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / dt / 1e9 / HBM_PEAK_GBS, "traffic": None,
                         "note": "algorithmic v2 in + v2 out over the host-timed call (all stages, one sync)"},
            "kernel": "k_v2_decode + merge pipeline + k_v2_encode", "stages_ms": {
                "v2_to_v1x": st_k["ms_v2_decode"], "merge": st_k["ms_v2_merge"], "v1x_to_v2": st_k["ms_v2_encode"]},
            "cpu_baseline": cpu}


def run_compact(a, eng, batch, tensors, dev, world):
    """Store-based compaction (ycompact_updates_v1_batch_device) of the same
    resident batch: every document's updates applied in order to a fresh Doc, then
    encode_state_as_update_v1.  Rank 0's shard; the CPU oracle on a bounded sample beside it."""
    import oracle
    t_b, t_u, t_d = tensors
    args = (t_b.data_ptr(), batch.n_bytes, t_u.data_ptr(), batch.n_updates, t_d.data_ptr(), batch.n_docs)
    eng.compact_device(*args)  # warm-up: scratch allocation
    runs = []
    for _ in range(2):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        r = eng.compact_device(*args)
        torch.cuda.synchronize(dev)
        runs.append(time.perf_counter() - t)
    st_k = eng.stats()
    _, _, st = r.to_host()
    dt = min(runs)
    cpu = None
    if not a.no_cpu_baseline and world == 1:
        k = min(batch.n_docs, 1000)
        s = batch.prefix(k)
        threads = min(16, os.cpu_count() or 1)  # the job's CPU share on the GPU box
        t = time.perf_counter()
        oracle.compact_batch(s.data, s.upd_off, s.doc_upd, threads=threads)
        ct = time.perf_counter() - t
        cpu = {"value": s.n_bytes / ct / 1e9, "unit": "GB/s", "docs_per_s": k / ct, "cores": threads, "kind": "port",
               "sample": f"oracle/yrs_oracle_store.c compact_updates_v1 on the first {k} documents"}
    # roofline of the dominant kernel: algorithmic bytes (input + output) over k_compact's
    # HIP-event time (the count pass and scans are k_compact_count_ms beside it)
    alg = batch.n_bytes + int(r.out_bytes)
    kms = max(float(st_k["ms_exact"]), 1e-6)
    return {"value": batch.n_bytes / dt / 1e9, "unit": "GB/s", "docs_per_s": batch.n_docs / dt, "ms": dt * 1e3,
            "k_compact_ms": st_k["ms_exact"], "count_scan_ms": st_k["ms_decode"],
            "out_bytes": int(r.out_bytes), "docs_device": int((st == 0).sum()),
            "docs_unsupported": int((st == 21).sum()),
            "roofline": {"bound": "hbm", "achieved": alg / (kms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None, "kernel": "k_compact",
                         "alg_bytes_per_launch": alg},
            "kernel": "k_compact_count + k_compact (lane per document)", "cpu_baseline": cpu}


def run_diff(a, rank, world, dev):
    """C5: diff_updates_v1 of compacted documents (the C2 merge outputs) against remote SVs."""
    import dist
    import workloads
    import ymerge
    docs, ops = a.docs or 100_000, a.ops or 1_000
    ids = dist.shard(world * docs, rank, world) if world > 1 else np.arange(docs, dtype=np.uint64)
    eng = ymerge.Engine(dev.index)
    # compact in chunks on the GPU (the merge outputs are the C5 documents)
    parts, chunk = [], 20_000
    for c0 in range(0, len(ids), chunk):
        b = workloads.text_docs(0, ops, ids=ids[c0:c0 + chunk])
        out, off, st = eng.merge_host(b.data, b.upd_off, b.doc_upd)
        assert not st.any(), "compaction failed"
        parts.append((out, off))
    data = np.concatenate([p[0] for p in parts])
    lens = np.concatenate([np.diff(p[1]) for p in parts]).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)

    def sv_fn(dd, oo):
        return eng.state_vector_host(dd, oo)
    db = workloads.compacted_docs(data, offs, sv_fn=sv_fn)
    t_b = torch.from_numpy(ymerge.padded(db.data)).to(dev)
    t_u = torch.from_numpy(db.upd_off.view(np.int64)).to(dev)
    t_s = torch.from_numpy(ymerge.padded(db.sv)).to(dev)
    t_so = torch.from_numpy(db.sv_off.view(np.int64)).to(dev)
    torch.cuda.synchronize(dev)

    def step():
        return eng.diff_device(t_b.data_ptr(), t_u.data_ptr(), t_s.data_ptr(), t_so.data_ptr(), db.n_docs)

    for _ in range(a.warmup):
        step()
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-stage HIP-event times from the same number of untimed steps (reading the stats is
    # not part of a step: the getter waits on the step's last event)
    kstats = []
    for _ in range(a.steps):
        res = step()
        kstats.append(eng.stats())
    out_bytes = res.out_bytes
    _, _, st = res.to_host()
    n_err = int((st != 0).sum())
    mean = lambda k: float(np.mean([s[k] for s in kstats]))  # noqa: E731
    ms_pipe = mean("ms_fast") + mean("ms_exact") + mean("ms_tail")
    bytes_in = db.n_bytes + int(db.sv_off[-1])
    allst = dist.gather_stats([db.n_docs, bytes_in, out_bytes, n_err, elapsed, ms_pipe], device=dev)
    if rank != 0:
        return None
    t_max = float(allst[:, 4].max())
    alg = bytes_in + out_bytes  # |update| + |remote SV| + |diff|
    achieved = alg / (ms_pipe * 1e-3) / 1e9
    cpu = None
    if not a.no_cpu_baseline and world == 1:
        import oracle
        model, nproc, share = host_cpu()
        per = max(1, bytes_in // max(1, db.n_docs))
        n_s = int(min(db.n_docs, max(16, a.cpu_seconds * 60e6 * share / per)))
        ub, uo = db.data[:int(db.upd_off[n_s])], db.upd_off[:n_s + 1]
        sb, so = db.sv[:int(db.sv_off[n_s])], db.sv_off[:n_s + 1]
        dt = timed_runs(lambda: oracle.diff_batch(ub, uo, sb, so, threads=share), 5)
        cpu = {"value": (len(ub) + len(sb)) / dt / 1e9, "unit": "GB/s", "cores": share, "kind": "port",
               "docs_per_s": n_s / dt, "cpu_model": model, "nproc": nproc,
               "sample": f"first {n_s} documents, oracle diff_updates_v1 restatement, {share} threads, "
                         f"median of 5 after 1 warm-up: {dt:.3f} s"}
    return {
        "metric": METRIC_DIFF, "value": float(allst[:, 1].sum()) * a.steps / t_max / 1e9, "unit": "GB/s",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": t_max / a.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "docs_per_s": float(allst[:, 0].sum()) * a.steps / t_max,
        "config": {"workload": f"C5: diff_updates_v1 of {docs} compacted docs per GPU (C2 merge outputs of {ops} "
                               "updates) against per-doc remote state vectors, inputs HBM-resident",
                   "docs_per_gpu": docs, "bytes_in_per_gpu": int(allst[0, 1]),
                   "bytes_out_per_gpu": int(allst[0, 2]), "error_docs": int(allst[:, 3].sum()),
                   "parallelism": f"doc-hash sharding x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic("c5"), "kernel": "k_plan+k_exec",
                     "kernel_ms": ms_pipe, "k_plan_ms": mean("ms_fast"), "replan_ms": mean("ms_exact"),
                     "k_exec_ms": mean("ms_tail"), "alg_bytes_per_launch": alg,
                     "stage_note": f"kernel_ms and the stage times are HIP-event means over {a.steps} "
                                   "separate untimed steps run after the timed loop (same batch)"},
        "cpu_baseline": cpu,
    }


def main():
    a = parse()
    import dist
    code = dist.relaunch(a.gpus, os.path.abspath(__file__), sys.argv[1:])  # before any GPU call
    if code is not None:
        sys.exit(code)
    rank, world, local = dist.init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    line = run_diff(a, rank, world, dev) if a.workload == "c5" else run_merge(a, rank, world, dev)
    if rank == 0:
        print(json.dumps(line))
    dist.finalize()


if __name__ == "__main__":
    main()
