"""Row-panel kNN against the whole n x n buffer (diagnostic, GPU box).

    python tools/panel_probe.py

Times the device graph (gll_graph: Gram + select + row build) at the utils.laplace shape
(60,250 x 128, k 50) with and without forced 1,024-row panels, and at 100,000 / 200,000 nodes
(d 64, k 10), where the n x n distances (40 / 160 GB) pass the 32 GiB line and panels of 8 GiB
are automatic.  Prints ms per graph and the workspace size.
"""
import ctypes as ct
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402


def feats(n, d, seed):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((64, d))
    return (c[rng.integers(0, 64, n)] + 0.6 * rng.standard_normal((n, d))).astype(np.float32)


def run(n, d, k, flags, reps=3):
    X = torch.from_numpy(feats(n, d, 1)).cuda()
    prob = GLL.make_problem(n, d, 0, 1, k, 0.0, "auto", flags=flags)
    wsb = _lib.lib().gll_workspace_bytes(ct.byref(prob))
    g = GLL.device_graph(X, k, "auto", flags=flags)   # warm-up
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        del g
        torch.cuda.synchronize()
        t = time.perf_counter()
        g = GLL.device_graph(X, k, "auto", flags=flags)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    idx = g["knn_idx"].cpu().numpy()
    print(f"n {n:>7} d {d:>4} k {k:>3} flags {flags:>6}: {1e3 * min(ts):9.1f} ms per graph "
          f"(workspace {wsb / 2**30:6.2f} GiB)", flush=True)
    return idx


if __name__ == "__main__":
    a = run(60250, 128, 50, 0)
    b = run(60250, 128, 50, _lib.FLAG_KNN_PANEL)
    print("kNN lists equal:", bool(np.array_equal(a, b)), flush=True)
    run(100_000, 64, 10, 0)
    run(200_000, 64, 10, 0, reps=1)
