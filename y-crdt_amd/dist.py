"""Multi-GPU plumbing for the batched engine (one process per GPU).

Documents are independent (yrs/src/alt.rs:15-81 take one document's data), so a
node partitions them by hash — document d belongs to rank splitmix64(d) % world
(workloads.shard_ids) — and every rank runs the whole pipeline on its shard with no
data-path collective.  torch.distributed ("nccl" = RCCL over xGMI on MI355X, "gloo"
on CPU for tests) carries only the barrier around the timed region and one
all-gather of a fixed-size per-rank stats vector after the batch.
"""
import os

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
