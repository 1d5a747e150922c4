"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo): SURVEY.md §8e.

Each rank owns an independent minibatch graph (seed = rank), computes its predictions with
the oracle (the GPU product path is exercised by the -m gpu tests), and all-gathers them the
way bench.py does; every rank must then hold every other rank's predictions bit-for-bit, and
the max-over-ranks timing reduction must agree on all ranks.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from graphlearninglayer_amd.parallel import PredictionGatherer, gather_predictions, shard_rank_seed
from graphlearninglayer_amd.synth import CONFIGS, one_hot, synth
from oracle import gll_oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard_predictions(rank):
    c = CONFIGS["plumbing"]
    X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=shard_rank_seed(0, rank))
    Y = one_hot(lab[: c["base"]])
    U, _ = gll_oracle.forward(X, Y, tau=0.07, epsilon=1.0, K=c["k"])
    return torch.from_numpy(np.ascontiguousarray(U, dtype=np.float32))


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        U = _shard_predictions(rank)
        full, work = gather_predictions(U, async_op=True)
        assert work is not None
        work.wait()
        t = torch.tensor([1.0 + rank], dtype=torch.float64)   # per-rank elapsed time
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        np.save(os.path.join(out_dir, f"r{rank}.npy"), full.numpy())
        np.save(os.path.join(out_dir, f"t{rank}.npy"), t.numpy())
    finally:
        dist.destroy_process_group()


def test_gather_predictions_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    m = CONFIGS["plumbing"]["batch"]
    expect = torch.cat([_shard_predictions(r) for r in range(world)]).numpy()
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npy")
        assert got.shape == (world * m, 10)
        np.testing.assert_array_equal(got, expect)
        assert float(np.load(tmp_path / f"t{r}.npy")[0]) == float(world)


def test_gather_predictions_single_process_is_identity():
    U = torch.arange(12, dtype=torch.float32).reshape(6, 2)
    out, work = gather_predictions(U)
    assert work is None and out is U


def test_shards_are_distinct_graphs():
    a, b = _shard_predictions(0), _shard_predictions(1)
    assert not torch.equal(a, b)


def _coalesced_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = PredictionGatherer(every=3)
        calls = [(_shard_predictions(rank) + s) for s in range(7)]   # 7 calls: groups 3, 3, 1
        for U in calls:
            g.add(U)
        g.wait()
        assert [t.shape for t in g.gathered] == [(world, 3, 64, 10), (world, 3, 64, 10),
                                                 (world, 1, 64, 10)]
        full = torch.cat([t.transpose(0, 1) for t in g.gathered])   # (calls, world, m, C)
        np.save(os.path.join(out_dir, f"c{rank}.npy"), full.numpy())
    finally:
        dist.destroy_process_group()


def test_coalesced_gatherer_world2(tmp_path):
    """bench.py's coalesced gather: every call's predictions of every rank, in call order."""
    world = 2
    mp.spawn(_coalesced_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    expect = np.stack([np.stack([(_shard_predictions(r) + s).numpy() for r in range(world)])
                       for s in range(7)])
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"c{r}.npy"), expect)


def test_coalesced_gatherer_single_process_is_noop():
    g = PredictionGatherer(every=2)
    g.add(torch.zeros(3, 2))
    g.wait()
    assert g.gathered == [] and g.pending == []


def _snapshot_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = PredictionGatherer(every=2)
        U = torch.full((4, 3), float(rank), requires_grad=True) * 1.0   # non-leaf, has a graph
        g.add(U)
        with torch.no_grad():
            U.add_(100.0)            # the CW pattern edits the output in place (adversarial.py:691)
        g.add(U)
        g.wait()
        (blk,) = g.gathered
        assert not blk.requires_grad
        np.save(os.path.join(out_dir, f"s{rank}.npy"), blk.numpy())
    finally:
        dist.destroy_process_group()


def test_gatherer_snapshots_calls_world2(tmp_path):
    """add() copies U at call time: an in-place edit afterwards changes only later calls."""
    world = 2
    mp.spawn(_snapshot_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        got = np.load(tmp_path / f"s{r}.npy")                     # (world, calls, 4, 3)
        for q in range(world):
            assert (got[q, 0] == q).all() and (got[q, 1] == q + 100.0).all()


def _bench(*args, env=None):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(v, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], env=e,
                       capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def test_bench_launches_its_own_ranks_dry_run():
    """`bench.py --gpus 2` (the driver's N>1 command without an outer torchrun) starts two
    ranks itself; rank 0 prints one line with n_gpus 2 and rank-ordered gathers."""
    rc, out, err = _bench("--gpus", "2", "--dry-run", "--steps", "17", "--warmup", "3")
    assert rc == 0, err[-2000:]
    assert out["n_gpus"] == 2 and out["steps"] == 17 and out["dry_run"] is True
    assert out["gather_check"] == "ok"
    assert out["config"]["parallelism"] == "dp2"
    # the self-proving fields of a scaling line: both ranks, as the process group saw them
    ranks = out["ranks"]
    assert [e["rank"] for e in ranks] == [0, 1]
    assert [e["local_rank"] for e in ranks] == [0, 1]
    assert all(e["world_size_seen"] == 2 for e in ranks)
    assert all(e["pci"] is None and e["current_device"] == -1 for e in ranks)   # CPU stand-in
    assert out["distinct_gpus"] is True


def test_distinct_devices_rejects_a_shared_gpu():
    from graphlearninglayer_amd.parallel import distinct_devices
    a = {"rank": 0, "local_rank": 0, "current_device": 0, "pci": "0000:05:00",
         "uuid_hash": "01", "world_size_seen": 2}
    b = dict(a, rank=1, local_rank=1, current_device=1, pci="0000:15:00", uuid_hash="02")
    assert distinct_devices([a, b])
    assert not distinct_devices([a, dict(b, pci="0000:05:00", uuid_hash="01")])
    assert not distinct_devices([a, dict(b, world_size_seen=1)])
    assert not distinct_devices([a, dict(b, rank=0)])


def test_bench_rejects_world_size_mismatch():
    rc, out, err = _bench("--gpus", "2", "--dry-run", env={"WORLD_SIZE": "1"})
    assert rc == 2 and out is None and "WORLD_SIZE=1" in err
