"""Multi-GPU data parallelism for the GLL path.

Independent minibatch graphs shard one per rank (one process per GPU, no cross-GPU graph
edges); the only collective is an all_gather of the per-rank predictions U (m x C) over
RCCL/xGMI ("nccl" backend on ROCm) -- or gloo on CPU for tests.  The gather is issued
asynchronously so it overlaps the backward of the same step.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_rank_seed(base_seed: int, rank: int) -> int:
    """Seed of the minibatch graph a rank owns (config 4 of BASELINE.json: seed = rank)."""
    return int(base_seed) + int(rank)


def gather_predictions(U: torch.Tensor, group=None, async_op: bool = True,
                       min_world: int = 2):
    """All-gather every rank's predictions into one (world * m) x C tensor.

    Returns (out, work): `out` is filled once `work.wait()` returns (work is None when
    async_op is False or the world has fewer than `min_world` ranks; `min_world=1` runs the
    collective even for one rank -- tests use it to drive RCCL on a one-GPU box)."""
    if not dist.is_available() or not dist.is_initialized():
        return U, None
    world = dist.get_world_size(group)
    if world < min_world:
        return U, None
    U = U.contiguous()
    out = torch.empty((world * U.shape[0],) + tuple(U.shape[1:]), dtype=U.dtype, device=U.device)
    work = dist.all_gather_into_tensor(out, U, group=group, async_op=async_op)
    return out, work


class PredictionGatherer:
    """All-gather of per-rank predictions coalesced over `every` calls (at NS a
    single gather moves 20 KB, so its ~10-30 us of launch and rendezvous latency, not bytes,
    is the cost; one gather per `every` calls amortises it).

    `add(U)` snapshots this call's U (detached, copied on the stream into slot i of the
    group's (every, m, C) block, so neither the autograd graph nor the saved workspace is
    kept alive and a later in-place edit of U -- adversarial.py:691 -- does not change what
    is gathered); the `every`-th call issues ONE asynchronous all_gather_into_tensor of the
    block; `flush()` issues it for a partial group.  Completed groups land in
    `self.gathered` as (world, calls, m, C) tensors in call order once `wait()` returns
    (only the newest `keep` of them when `keep` is set).  With fewer than `min_world` ranks
    (default 2; or no process group) it is a no-op that records nothing: `min_world=1` runs
    the collective at world size 1 (tests drive RCCL on a one-GPU box that way)."""

    def __init__(self, every: int = 8, group=None, keep=None, min_world: int = 2):
        self.every = max(1, int(every))
        self.group = group
        self.keep = keep
        self.min_world = max(1, int(min_world))
        self._block = None      # (every, m, C) snapshots of the current group
        self._fill = 0
        self.inflight = []      # (out tensor, work)
        self.gathered = []

    @property
    def pending(self):
        return [] if self._block is None else list(self._block[: self._fill])

    def _active(self) -> bool:
        return (dist.is_available() and dist.is_initialized()
                and dist.get_world_size(self.group) >= self.min_world)

    def add(self, U: torch.Tensor) -> None:
        if not self._active():
            return
        U = U.detach()
        b = self._block
        if b is not None and (b.shape[1:] != U.shape or b.dtype != U.dtype
                              or b.device != U.device):
            self.flush()
            b = None
        if b is None:
            # a fresh block per group: the previous one may still be read by its collective
            b = self._block = torch.empty((self.every,) + tuple(U.shape), dtype=U.dtype,
                                          device=U.device)
            self._fill = 0
        b[self._fill].copy_(U)
        self._fill += 1
        if self._fill >= self.every:
            self.flush()

    def _host_staged(self, t: torch.Tensor) -> bool:
        # gloo moves host memory: device blocks go through a host copy (the diagnostic that
        # runs several ranks on one GPU, bench.py --share-gpu; RCCL is the production path)
        return t.is_cuda and dist.get_backend(self.group) == "gloo"

    def flush(self) -> None:
        if self._block is None or self._fill == 0:
            return
        world = dist.get_world_size(self.group)
        block = self._block[: self._fill]
        self._block, self._fill = None, 0
        dev = block.device
        if self._host_staged(block):
            block = block.cpu()
        # concatenated along dim 0 (the layout every backend accepts), viewed per rank below
        out = torch.empty((world * block.shape[0],) + tuple(block.shape[1:]), dtype=block.dtype,
                          device=block.device)
        work = dist.all_gather_into_tensor(out, block, group=self.group, async_op=True)
        self.inflight.append((out.view((world,) + tuple(block.shape)), work, dev))

    def wait(self) -> None:
        """Flush the partial group and wait for every issued gather."""
        self.flush()
        for out, work, dev in self.inflight:
            work.wait()
            self.gathered.append(out.to(dev))
        self.inflight = []
        if self.keep is not None and len(self.gathered) > self.keep:
            del self.gathered[: len(self.gathered) - self.keep]


def _pci_fields(dev) -> tuple:
    """(domain, bus, device, uuid hash) of a GPU, all -1 for a CPU rank."""
    if dev is None or dev.type != "cuda":
        return (-1, -1, -1, -1)
    import hashlib
    p = torch.cuda.get_device_properties(dev)
    uu = int.from_bytes(hashlib.sha256(str(getattr(p, "uuid", "")).encode()).digest()[:7], "little")
    return (int(getattr(p, "pci_domain_id", -1)), int(getattr(p, "pci_bus_id", -1)),
            int(getattr(p, "pci_device_id", -1)), uu)


def rank_identity(dev=None, coll=None, group=None) -> list:
    """Every rank's (rank, LOCAL_RANK, current device, PCI address, world size it sees), as the
    process group itself gathers them: one tiny all_gather, called outside any timed region.

    This makes a scaling run self-proving (each of N ranks on its own GPU, RCCL seeing N
    ranks).  `dev` is the rank's GPU (None: a CPU rank), `coll` the device the collective
    moves tensors on (the GPU for RCCL, the CPU for gloo).  Without a process group it
    returns this process alone."""
    import os
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cur = torch.cuda.current_device() if dev is not None and dev.type == "cuda" else -1
    if dist.is_available() and dist.is_initialized():
        rank, world = dist.get_rank(group), dist.get_world_size(group)
    else:
        rank, world = 0, 1
    mine = torch.tensor([rank, local, cur, *_pci_fields(dev), world], dtype=torch.int64)
    if world > 1 or (dist.is_available() and dist.is_initialized()):
        mine = mine.to(coll if coll is not None else "cpu")
        allr = torch.empty(world * mine.numel(), dtype=torch.int64, device=mine.device)
        dist.all_gather_into_tensor(allr, mine, group=group)
        rows = allr.view(world, -1).cpu().tolist()
    else:
        rows = [mine.tolist()]
    out = []
    for r, lr, cd, dom, bus, pdev, uu, ws in rows:
        out.append({"rank": r, "local_rank": lr, "current_device": cd,
                    "pci": (f"{dom:04x}:{bus:02x}:{pdev:02x}" if bus >= 0 else None),
                    "uuid_hash": (f"{uu:014x}" if uu >= 0 else None),
                    "world_size_seen": ws})
    return out


def distinct_devices(ident: list) -> bool:
    """True when no two ranks report the same GPU (PCI address and device UUID) and every rank
    saw as many ranks as there are entries."""
    gpus = [(e["pci"], e["uuid_hash"]) for e in ident if e["pci"] is not None]
    sizes = {e["world_size_seen"] for e in ident}
    ranks = sorted(e["rank"] for e in ident)
    return (len(set(gpus)) == len(gpus) and sizes == {len(ident)}
            and ranks == list(range(len(ident))))
