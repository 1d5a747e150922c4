"""Per-kernel times of one fwd+bwd at the ns / fullysup / stress shapes, single and batched
(diagnostic A/B, run on the GPU box; pick the library with GLL_LIB_PATH).

    python tools/select_ab.py [--cases ns:1,ns:64,fullysup:1,fullysup:64,stress:1] [--tag T]

Every kernel of the chain is timed by the events in its dispatch packet (_lib.prof_*); the
forward output U is saved under gpurun_out/select_ab_<tag>_<case>.npy, and when a file of the
tag given by --against exists its max relative difference is printed.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cases", default="ns:1,ns:64,fullysup:1,fullysup:64,stress:1")
ap.add_argument("--tag", default="new")
ap.add_argument("--against", default="")
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
os.makedirs("gpurun_out", exist_ok=True)
GLL._ext_mod = False   # the Python Function onto _lib's library (the C++ node links libgll.so)
print("library:", _lib.LIB_PATH, "GLL_SEL_DIAG", os.environ.get("GLL_SEL_DIAG", "0"), flush=True)
names = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)]
lap = GLL.LaplaceLearningSparseHard.apply
for case in a.cases.split(","):
    cfg, B = case.split(":")
    B = int(B)
    c = CONFIGS[cfg]
    eps = "auto" if cfg == "stress" else 1.0
    Xs, Ys = [], []
    for g in range(min(B, 8)):
        X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=g)
        Xs.append(X)
        Ys.append(one_hot(lab[: c["base"]]))
    reps = (B + len(Xs) - 1) // len(Xs)
    if B == 1:
        Xb = torch.from_numpy(Xs[0]).cuda().requires_grad_(True)
        Yb = torch.from_numpy(Ys[0]).cuda()
        G = torch.from_numpy(seeded_gbar(c["batch"], 10, 1234)).cuda()
    else:
        Xb = torch.from_numpy(np.concatenate([np.stack(Xs)] * reps)[:B]).cuda().requires_grad_(True)
        Yb = torch.from_numpy(np.concatenate([np.stack(Ys)] * reps)[:B]).cuda()
        G = torch.from_numpy(np.stack([seeded_gbar(c["batch"], 10, 1234 + g) for g in range(B)])).cuda()

    def step():
        U = lap(Xb, Yb, 0.07, eps, c["k"])
        return U, torch.autograd.grad(U, Xb, G)[0]

    for _ in range(3):
        U, gx = step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    for q in range(_lib.K_COUNT):
        _lib.prof_enable(q, 1)
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    parts = []
    for q in range(_lib.K_COUNT):
        ms, cnt = _lib.prof_read(q)
        _lib.prof_enable(q, 0)
        if cnt:
            parts.append(f"{names[q]} {1e3 * ms / cnt:.1f}")
    U, gx = step()
    Un = U.detach().double().cpu().numpy()
    gn = gx.double().cpu().numpy()
    np.save(f"gpurun_out/select_ab_{a.tag}_{cfg}_{B}.npy", Un)
    diff = ""
    ref = f"gpurun_out/select_ab_{a.against}_{cfg}_{B}.npy"
    if a.against and os.path.exists(ref):
        R = np.load(ref)
        diff = f" | dU vs {a.against} {np.abs(Un - R).max() / np.abs(R).max():.1e}"
    print(f"{cfg} B={B}: {1e6 * wall:.1f} us/call | " + ", ".join(parts) + f" us{diff}", flush=True)
    del Xb, Yb, G, U, gx
    torch.cuda.empty_cache()
