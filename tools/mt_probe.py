"""Step time through apply + autograd.grad with torch's autograd multithreading on and off
(diagnostic, GPU box).  With it off the engine runs the CUDA backward on the calling thread
instead of handing it to its per-device worker thread."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

c = CONFIGS["ns"]
X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
X = torch.from_numpy(X_np).cuda().requires_grad_(True)
Y = torch.from_numpy(one_hot(lab[: c["base"]])).cuda()
g = torch.from_numpy(seeded_gbar(c["batch"], 10, 1234)).cuda()
lap = GLL.LaplaceLearningSparseHard.apply


def run(steps):
    for _ in range(steps):
        U = lap(X, Y, 0.07, 1.0, c["k"])
        torch.autograd.grad(U, X, g)


for mode in [True, False, True, False]:
    with torch.autograd.set_multithreading_enabled(mode):
        run(20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(300)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 300
    print(f"multithreading={mode}: {1e6 * dt:.1f} us/step ({1 / dt:.0f} calls/s)", flush=True)
