"""Benchmark: batched merge_updates_v1 on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--docs D] [--ops O]

Workload (BASELINE.json configs[1]): per GPU 10,000 synthetic YText documents x
1,000 single-op v1 updates (1-4 synced clients, 80/20 insert/delete), inputs
resident in HBM before the timed region.  One step = one full batched
merge_updates_v1 over the GPU's shard (validate/count, scratch plan, size plan,
scan, write).  For N > 1 (torch.distributed.run, one rank per GPU) documents are
sharded by splitmix64(doc_id) % N with no data-path collective; RCCL is used for
the barrier, the max-over-ranks time and a per-shard stats gather.

Prints ONE JSON line (rank 0).  `value` = input GB/s over all ranks; docs/s,
roofline of the dominant kernel (HIP-event timed on the engine's stream) and the
CPU baseline (the oracle, literal yrs algorithm, on a bounded sample, rank 0,
N=1) ride along.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "y-crdt_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "input GB/s + docs compacted/sec, batched merge_updates_v1 @ 1/2/4/8 GPUs"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--docs", type=int, default=10_000, help="documents per GPU")
    ap.add_argument("--ops", type=int, default=1_000, help="updates per document")
    ap.add_argument("--cpu-sample", type=int, default=10_000, help="docs in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def pmc_traffic():
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3 PMC pass, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        try:
            with open(p) as f:
                return json.load(f).get("traffic_bytes_per_launch")
        except Exception:
            return None
    return None


def main():
    a = parse()
    import dist
    rank, world, local = dist.init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import workloads
    import ymerge

    # ---- shard: doc-hash partition of world * docs global documents
    ids = dist.shard(world * a.docs, rank, world) if world > 1 else np.arange(a.docs, dtype=np.uint64)
    batch = workloads.text_docs(len(ids), a.ops, ids=ids)
    t_b = torch.from_numpy(batch.data).to(dev)
    t_u = torch.from_numpy(batch.upd_off.view(np.int64)).to(dev)
    t_d = torch.from_numpy(batch.doc_upd.view(np.int64)).to(dev)
    torch.cuda.synchronize(dev)
    eng = ymerge.Engine(local)

    def step():
        return eng.merge_device(t_b.data_ptr(), batch.n_bytes, t_u.data_ptr(), batch.n_updates, t_d.data_ptr(),
                                batch.n_docs)

    for _ in range(a.warmup):
        step()
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    kstats = []
    for _ in range(a.steps):
        res = step()
        kstats.append(eng.stats())
    torch.cuda.synchronize(dev)
    dist.barrier()
    elapsed = time.perf_counter() - t0

    out_bytes = res.out_bytes
    _, _, st = res.to_host()
    n_err = int((st != 0).sum())
    ms_merge = float(np.mean([s["ms_fast"] for s in kstats]))
    ms_decode = float(np.mean([s["ms_decode"] for s in kstats]))
    ms_kernel = ms_merge + ms_decode
    ms_exact = float(np.mean([s["ms_exact"] for s in kstats]))
    docs_exact = int(kstats[-1]["docs_exact"])
    allst = dist.gather_stats([batch.n_docs, batch.n_bytes, out_bytes, n_err, elapsed, ms_kernel], device=dev)
    if rank != 0:
        dist.finalize()
        return

    t_max = float(allst[:, 4].max())
    docs_total = float(allst[:, 0].sum()) * a.steps
    bytes_in_total = float(allst[:, 1].sum()) * a.steps
    ms_step = t_max / a.steps * 1e3
    value = bytes_in_total / t_max / 1e9
    # roofline of the merge kernel pair (k_decode -> k_fast_merge; together they are the path,
    # neither does the merge alone), algorithmic bytes = input + output
    alg_bytes = batch.n_bytes + out_bytes
    achieved = alg_bytes / (ms_kernel * 1e-3) / 1e9
    traffic = pmc_traffic()

    cpu = None
    if not a.no_cpu_baseline and world == 1:
        import oracle
        n_s = min(a.cpu_sample, batch.n_docs)
        sample = batch.subset(range(n_s))
        threads = min(16, os.cpu_count() or 1)
        t = time.perf_counter()
        oracle.merge_batch(sample.data, sample.upd_off, sample.doc_upd, mode=0, threads=threads)
        dt = time.perf_counter() - t
        cpu = {"value": sample.n_bytes / dt / 1e9, "unit": "GB/s", "cores": threads, "kind": "port",
               "docs_per_s": n_s / dt,
               "sample": f"first {n_s} docs of the same workload ({sample.n_bytes} B), oracle literal yrs loop "
                         f"(per-iteration decoder re-sort, DS re-squash), {threads} threads, {dt:.2f} s wall"}

    line = {
        "metric": METRIC, "value": value, "unit": "GB/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "docs_per_s": docs_total / t_max,
        "config": {"workload": f"C2: {a.docs} synthetic YText docs x {a.ops} single-op v1 updates per GPU, "
                               "batched merge_updates_v1, inputs HBM-resident",
                   "docs_per_gpu": a.docs, "updates_per_doc": a.ops,
                   "bytes_in_per_gpu": int(allst[0, 1]), "bytes_out_per_gpu": int(allst[0, 2]),
                   "parallelism": f"doc-hash sharding x{world}", "error_docs": int(allst[:, 3].sum())},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "k_decode+k_fast_merge", "kernel_ms": ms_kernel, "k_decode_ms": ms_decode,
                     "k_fast_merge_ms": ms_merge, "exact_path_ms": ms_exact,
                     "docs_exact_path": docs_exact, "alg_bytes_per_launch": alg_bytes},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))
    dist.finalize()


if __name__ == "__main__":
    main()
