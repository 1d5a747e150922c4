"""Per-kernel time of the batched entry point vs B at NS (diagnostic, GPU box)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

cfg = os.environ.get("PROBE_CFG", "ns")
c = CONFIGS[cfg]
eps = os.environ.get("PROBE_EPS", "1.0")
eps = eps if eps == "auto" else float(eps)
dev = torch.device("cuda", 0)
names = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)]
Xs, Ys = [], []
for g in range(8):
    X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=g)
    Xs.append(X)
    Ys.append(one_hot(lab[: c["base"]]))
for B in [int(v) for v in os.environ.get("PROBE_B", "1,8,32,64,128,256").split(",")]:
    reps = (B + 7) // 8
    Xb = torch.from_numpy(np.concatenate([np.stack(Xs)] * reps)[:B]).to(dev).requires_grad_(True)
    Yb = torch.from_numpy(np.concatenate([np.stack(Ys)] * reps)[:B]).to(dev)
    G = torch.from_numpy(np.stack([seeded_gbar(c["batch"], 10, g) for g in range(B)])).to(dev)

    def step():
        U = GLL.LaplaceLearningSparseHard.apply(Xb, Yb, 0.07, eps, c["k"])
        return torch.autograd.grad(U, Xb, G)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = 10
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    for q in range(_lib.K_COUNT):
        _lib.prof_enable(q, 1)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    parts = []
    for q in range(_lib.K_COUNT):
        ms, cnt = _lib.prof_read(q)
        _lib.prof_enable(q, 0)
        if cnt:
            parts.append(f"{names[q]}={1e3 * ms / cnt:.1f}")
    print(f"B={B:4d} step {1e6 * wall:9.1f} us ({1e6 * wall / B:6.2f} us/graph, "
          f"{B / wall:9.0f} calls/s): " + " ".join(parts), flush=True)
