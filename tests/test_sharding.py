"""Multi-process path on CPU (gloo, world_size 2): the doc-hash partition used by
bench.py / dist.py is disjoint and complete, every rank merges only its shard, and
the per-rank stats all-gather + max-over-ranks reduction reproduce the single-process
totals.  The merge in each rank is the CPU oracle in the CPU test, and the HIP engine
(ymerge.Engine on cuda:0, both ranks sharing the box's one GPU) in the `gpu` variant."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

N_DOCS, OPS = 48, 60


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q, use_gpu=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "y-crdt_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import dist
    import oracle
    import workloads
    r, w, _ = dist.init_from_env("gloo")
    ids = dist.shard(N_DOCS, r, w)
    b = workloads.text_docs(len(ids), OPS, ids=ids)
    if use_gpu:
        import ymerge
        eng = ymerge.Engine(0)
        out, off, st = eng.merge_host(b.data, b.upd_off, b.doc_upd)
        out = out.tobytes()
        eng.close()
    else:
        out, off, st = oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=2)
    per_doc = {int(ids[k]): out[int(off[k]):int(off[k + 1])] for k in range(len(ids))}
    dist.barrier()
    stats = dist.gather_stats([len(ids), b.n_bytes, len(out), int((st != 0).sum()), 0.1 * (r + 1)])
    gathered = [None] * w
    torch.distributed.all_gather_object(gathered, per_doc)
    if r == 0:
        q.put((stats, gathered))
    dist.finalize()


@pytest.mark.parametrize("use_gpu", [False, pytest.param(True, marks=pytest.mark.gpu)])
def test_two_rank_sharded_merge(oracle, use_gpu):
    import workloads
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q, use_gpu)) for r in range(world)]
    for p in procs:
        p.start()
    stats, gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # partition: disjoint and complete
    keys = [set(g) for g in gathered]
    assert not (keys[0] & keys[1])
    assert keys[0] | keys[1] == set(range(N_DOCS))
    # shard sizes as the hash partition says
    for r in range(world):
        assert len(workloads.shard_ids(N_DOCS, r, world)) == int(stats[r, 0])
    # each document's output equals the single-process merge of that document
    full = workloads.text_docs(N_DOCS, OPS, ids=np.arange(N_DOCS, dtype=np.uint64))
    out, off, st = oracle.merge_batch(full.data, full.upd_off, full.doc_upd, mode=1, threads=2)
    merged = {**gathered[0], **gathered[1]}
    for d in range(N_DOCS):
        assert merged[d] == out[int(off[d]):int(off[d + 1])]
    # stats reduction: totals over ranks, time = max over ranks
    assert int(stats[:, 0].sum()) == N_DOCS
    assert int(stats[:, 1].sum()) == full.n_bytes
    assert int(stats[:, 2].sum()) == len(out)
    assert stats[:, 4].max() == pytest.approx(0.2)


_LAUNCH_SCRIPT = r'''
import json, os, sys
sys.path.insert(0, {ydir!r})
import dist
import torch
code = dist.relaunch(int(sys.argv[1]), os.path.abspath(__file__), sys.argv[1:], need_gpus=False)
if code is not None:
    sys.exit(code)
r, w, local = dist.init_from_env("gloo")
st = dist.gather_stats([r, w, local])
if r == 0:
    print(json.dumps({{"world": w, "ranks": sorted(int(x) for x in st[:, 0])}}))
dist.finalize()
'''


def test_bench_gpus_flag_starts_ranks(tmp_path):
    """`bench.py --gpus N` without WORLD_SIZE starts N ranks (dist.relaunch, the launcher path
    bench.py uses before any GPU call); with WORLD_SIZE set, a mismatching --gpus fails."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "launch.py"
    script.write_text(_LAUNCH_SCRIPT.format(ydir=os.path.join(root, "y-crdt_amd")))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, str(script), "2"], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line == {"world": 2, "ranks": [0, 1]}
    bad = subprocess.run([sys.executable, str(script), "2"], env=dict(env, WORLD_SIZE="1"), capture_output=True,
                         text=True, timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE=1" in bad.stderr


def test_visible_gpus_without_hip(monkeypatch):
    """dist.visible_gpus counts GPUs from the KFD topology and the visibility variables only (no
    HIP call in the parent of the rank processes)."""
    import dist
    n = dist.visible_gpus()
    assert n >= 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert dist.visible_gpus() == min(n, 1)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert dist.visible_gpus() == 0
