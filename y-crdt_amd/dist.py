"""Multi-GPU plumbing for the batched engine (one process per GPU).

Documents are independent (yrs/src/alt.rs:15-81 take one document's data), so a
node partitions them by hash — document d belongs to rank splitmix64(d) % world
(workloads.shard_ids) — and every rank runs the whole pipeline on its shard with no
data-path collective.  torch.distributed ("nccl" = RCCL over xGMI on MI355X, "gloo"
on CPU for tests) carries only the barrier around the timed region and one
all-gather of a fixed-size per-rank stats vector after the batch.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import torch

import workloads


def init_from_env(backend=None):
    """(rank, world, local_rank); initialises the process group when WORLD_SIZE > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not torch.distributed.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        torch.distributed.init_process_group(backend, **kw)
    return rank, world, local


def visible_gpus():
    """GPUs this process may use, without initialising HIP: the GPU nodes of the KFD topology
    (/sys/class/kfd/kfd/topology/nodes/*/properties with simd_count > 0), limited by
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    for line in f:
                        k, _, v = line.partition(" ")
                        if k == "simd_count" and int(v) > 0:
                            n += 1
                            break
            except (OSError, ValueError):
                pass
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def relaunch(n, script, argv, need_gpus=True):
    """Make `python script --gpus n` mean n ranks on this node.

    Inside a torch.distributed.run rank (WORLD_SIZE set) the requested count must equal the
    world size; otherwise, for n > 1, the n rank processes are started as ONE child
    (`python -m torch.distributed.run --nproc-per-node n ...`, rendezvous on 127.0.0.1) and
    its exit code is returned: the caller exits with it.  The GPUs are counted from the KFD
    topology (visible_gpus), so this parent never initialises the HIP runtime.  Returns None
    when this process should run the work itself."""
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if n is not None and n != world:
            raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}: launch one rank per GPU")
        return None
    if n is None or n <= 1:
        return None
    if need_gpus:
        have = visible_gpus()
        if have < n:
            raise SystemExit(f"--gpus {n} but only {have} GPU(s) visible")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", script] + list(argv)
    return subprocess.call(cmd)


def shard(n_total, rank, world):
    """Global document ids owned by `rank` (doc-hash partition, disjoint and complete)."""
    return workloads.shard_ids(n_total, rank, world)


def gather_stats(values, device=None):
    """All-gather one float64 vector per rank -> array [world, len(values)]."""
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return t.cpu().numpy()[None, :]
    out = [torch.zeros_like(t) for _ in range(torch.distributed.get_world_size())]
    torch.distributed.all_gather(out, t)
    return torch.stack(out).cpu().numpy()


def barrier():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.barrier()


def finalize():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
