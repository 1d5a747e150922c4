"""Host cost of the pieces of one step (diagnostic, GPU box): Python wrapper, C++ node
forward, autograd backward, with the GPU kept busy so only enqueue cost is seen."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL  # noqa: E402
from graphlearninglayer_amd import _gll_torch as ext  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

c = CONFIGS["ns"]
dev = torch.device("cuda", 0)
X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
X = torch.from_numpy(X_np).to(dev).requires_grad_(True)
Y = torch.from_numpy(one_hot(lab[: c["base"]])).to(dev)
g = torch.from_numpy(seeded_gbar(c["batch"], 10)).to(dev)
sink = GLL._sink(dev)[0].data_ptr()


def timeit(label, fn, n=400):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    print(f"{label:44s} {1e6 * t:7.1f} us enqueue", flush=True)


timeit("GLL.apply (python wrapper + node)", lambda: GLL.LaplaceLearningSparseHard.apply(X, Y, 0.07, 1.0, 10))
timeit("ext.laplace_learning (node only)", lambda: ext.laplace_learning(X, Y, 0.07, 1.0, 10, 1000, 1e-6, sink))
Xn = X.detach()
timeit("ext.laplace_learning, no grad (no node)", lambda: ext.laplace_learning(Xn, Y, 0.07, 1.0, 10, 1000, 1e-6, sink))
U = GLL.LaplaceLearningSparseHard.apply(X, Y, 0.07, 1.0, 10)


def fb():
    U = ext.laplace_learning(X, Y, 0.07, 1.0, 10, 1000, 1e-6, sink)
    torch.autograd.grad(U, X, g)


timeit("node fwd + autograd.grad", fb)


def fb2():
    U = ext.laplace_learning(X, Y, 0.07, 1.0, 10, 1000, 1e-6, sink)
    U.backward(g)


timeit("node fwd + U.backward (accumulates X.grad)", fb2)
timeit("torch.empty x2 (allocator)", lambda: (torch.empty(4_400_000, dtype=torch.uint8, device=dev),
                                            torch.empty(500, 10, dtype=torch.float64, device=dev)))
