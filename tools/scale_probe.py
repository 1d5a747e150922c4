"""Kernel time vs problem size (diagnostic, GPU box): latency- or throughput-bound?

For n in a sweep, runs the device graph build (gll_graph: Gram MFMA, select, row build) and
one forward+backward, bracketing every launch with HIP events via the library's profiling
hook, and prints the average microseconds per kernel.
"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import one_hot, seeded_gbar, synth  # noqa: E402

dev = torch.device("cuda", 0)
names = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)]
d = int(os.environ.get("PROBE_D", "512"))
k = int(os.environ.get("PROBE_K", "10"))
for n in [int(v) for v in os.environ.get("PROBE_N", "512,1000,2000,4096,8192").split(",")]:
    base = n // 2
    X_np, lab = synth(base, n - base, d, r=1.0, seed=0)
    X = torch.from_numpy(X_np).to(dev).requires_grad_(True)
    Y = torch.from_numpy(one_hot(lab[:base])).to(dev)
    g = torch.from_numpy(seeded_gbar(n - base, 10)).to(dev)
    lap = GLL.LaplaceLearningSparseHard.apply
    for _ in range(5):
        torch.autograd.grad(lap(X, Y, 0.07, 1.0, k), X, g)
    torch.cuda.synchronize()
    for q in range(_lib.K_COUNT):
        _lib.prof_enable(q, 1)
    reps = 20
    for _ in range(reps):
        torch.autograd.grad(lap(X, Y, 0.07, 1.0, k), X, g)
    torch.cuda.synchronize()
    parts = []
    for q in range(_lib.K_COUNT):
        ms, cnt = _lib.prof_read(q)
        _lib.prof_enable(q, 0)
        if cnt:
            parts.append(f"{names[q]}={1e3 * ms / cnt:.1f}")
    flops = 2.0 * n * n * d
    print(f"n={n} d={d} k={k}: " + " ".join(parts) + f"  (gram {flops / 1e9:.2f} GFLOP)", flush=True)
