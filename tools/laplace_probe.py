"""utils.laplace at the reference's evaluation size (diagnostic, GPU box):
n = 250 labeled + 50,000 unlabeled train + 10,000 test, d = 128, k = 50, eps = 1, tau = 1e-8."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib, utils  # noqa: E402
from graphlearninglayer_amd.synth import synth  # noqa: E402

for nl, nu, d in [(250, 20000, 128), (250, 60000, 128)]:
    X, labels = synth(nl, nu, d, C=10, r=1.0, seed=3)
    Xd = torch.from_numpy(X).cuda()
    utils.laplace(Xd[:2000], labels[:nl])          # warm-up (kernels, allocator)
    torch.cuda.synchronize()
    # the first call at a size pays the caching allocator's hipMalloc of the n^2 D2 workspace
    # (14.5 GB at 60k); the reference re-evaluates every --plot_freq_ss epochs at one size, so
    # the steady state is the later calls (the allocator keeps the block)
    for rep in range(3):
        t0 = time.perf_counter()
        g = GLL.device_graph(Xd, 50, 1.0)
        torch.cuda.synchronize()
        t_graph = time.perf_counter() - t0
        del g
        t0 = time.perf_counter()
        U = utils.laplace(Xd, labels[:nl], knn_num=50, epsilon=1.0, tau=1e-8)
        t_all = time.perf_counter() - t0
        acc = 100.0 * np.mean(U.argmax(1) == labels[nl:])
        print(f"n={nl + nu} d={d} k=50 {'first' if rep == 0 else 'warm '}: laplace "
              f"{t_all * 1e3:.1f} ms (graph alone {t_graph * 1e3:.1f} ms), GL accuracy {acc:.2f}%",
              flush=True)
    del Xd
    torch.cuda.empty_cache()
