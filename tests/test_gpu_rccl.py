"""The sharded path's collective on the GPU (BASELINE config 4).

bench.py --gpus N opens an "nccl" (RCCL) process group with `device_id` and gathers every rank's
predictions U with one asynchronous all_gather_into_tensor per GATHER_EVERY calls
(parallel.PredictionGatherer).  A one-GPU box cannot run two RCCL ranks, so this test opens the
same group at world size 1 -- the same init call as bench.py, the same collective on device
tensors -- with the gatherer told to gather at world 1 (`min_world=1`), and checks that every
call's U comes back in call order.  The world-2 semantics are covered over gloo on the CPU
(tests/test_parallel_cpu.py).  The per-minibatch graph it shards is FullySup.py:154-156's.
"""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_gather_of_predictions_at_world_one():
    from graphlearninglayer_amd import GLL
    from graphlearninglayer_amd.parallel import PredictionGatherer, gather_predictions
    from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth
    assert not dist.is_initialized()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # bench.py's init (bench.py main): backend "nccl" = RCCL on ROCm, bound to the rank's device
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        c = CONFIGS["ns"]
        X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
        Xd = torch.from_numpy(X).to(dev).requires_grad_(True)
        Y = torch.from_numpy(one_hot(lab[: c["base"]])).to(dev)
        g = torch.from_numpy(seeded_gbar(c["batch"], 10, 3)).to(dev)
        gatherer = PredictionGatherer(every=2, min_world=1)
        Us = []
        for t in range(5):
            U = GLL.LaplaceLearningSparseHard.apply(Xd, Y, 0.07, 1.0, c["k"])
            gatherer.add(U)                      # snapshots U on the stream
            Us.append(U.detach().clone())
            (gx,) = torch.autograd.grad(U, Xd, g)
            U.detach().mul_(1.0 + t)             # an in-place edit after add (adversarial.py:691)
        gatherer.wait()                          # two full groups and a partial one
        assert [tuple(b.shape) for b in gatherer.gathered] == [(1, 2) + tuple(Us[0].shape)] * 2 + \
            [(1, 1) + tuple(Us[0].shape)]
        got = torch.cat([b[0] for b in gatherer.gathered])
        assert got.device == dev and got.dtype == torch.float64
        for t in range(5):
            assert torch.equal(got[t], Us[t]), t
        # the per-call form
        out, work = gather_predictions(Us[0], min_world=1)
        work.wait()
        assert out.shape == Us[0].shape and torch.equal(out, Us[0])
        assert np.isfinite(gx.cpu().numpy()).all()
        # bench.py's self-proving fields (rank_identity: one all_gather over RCCL)
        from graphlearninglayer_amd.parallel import distinct_devices, rank_identity
        ident = rank_identity(dev, dev)
        assert len(ident) == 1 and ident[0]["rank"] == 0 and ident[0]["world_size_seen"] == 1
        assert ident[0]["current_device"] == 0
        p = torch.cuda.get_device_properties(dev)
        assert ident[0]["pci"] == f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
        assert ident[0]["uuid_hash"] is not None
        assert distinct_devices(ident)
        print("rank identity:", ident)
    finally:
        dist.destroy_process_group()
