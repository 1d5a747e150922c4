"""Why a kernel times differently through the torch apply than through the raw C ABI (diagnostic,
GPU box).  Same NS graphs, same kernels; per-kernel mean launch time (events in the dispatch
packet) under:
  abi          gll_forward_batched + gll_backward_batched, one workspace, prof on every kernel
  abi_cgonly   the same, prof on the CG kernel only (as bench.py's batched line)
  abi_fresh    a fresh torch.empty workspace per call (as the apply allocates one)
  apply        LaplaceLearningSparseHard.apply + autograd.grad, prof on every kernel
  apply_cgonly the same, prof on the CG kernel only
    PROBE_B=64 python tools/path_probe.py
"""
import ctypes as ct
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

B = int(os.environ.get("PROBE_B", "64"))
cfg = os.environ.get("PROBE_CFG", "ns")
c = CONFIGS[cfg]
n, m, d, k = c["base"] + c["batch"], c["batch"], c["d"], c["k"]
lib = _lib.lib()
names = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)]
cg = names.index("cg_kernel")
Xs, Ys = [], []
for g in range(min(B, 8)):
    X, lab = synth(c["base"], m, d, r=c["r"], seed=g)
    Xs.append(X)
    Ys.append(one_hot(lab[: c["base"]]))
reps = (B + len(Xs) - 1) // len(Xs)
Xb = torch.from_numpy(np.concatenate([np.stack(Xs)] * reps)[:B]).cuda().contiguous()
Yb = torch.from_numpy(np.concatenate([np.stack(Ys)] * reps)[:B]).cuda().contiguous()
G = torch.from_numpy(np.stack([seeded_gbar(m, 10, 1234 + g) for g in range(B)])).cuda()
s = torch.cuda.current_stream().cuda_stream
prob = GLL.make_problem(n, d, c["base"], 10, k, 0.07, 1.0)
wb = lib.gll_workspace_bytes(ct.byref(prob))
ws_once = torch.zeros(wb * B, dtype=torch.uint8, device="cuda")
U = torch.empty(B, m, 10, dtype=torch.float64, device="cuda")
gx = torch.empty(B, n, d, dtype=torch.float32, device="cuda")


def abi(fresh):
    def run():
        ws = torch.empty(wb * B, dtype=torch.uint8, device="cuda") if fresh else ws_once
        _lib.check(lib.gll_forward_batched(ct.byref(prob), B, Xb.data_ptr(), Yb.data_ptr(), 0,
                                           ws.data_ptr(), U.data_ptr(), s), "fwd")
        _lib.check(lib.gll_backward_batched(ct.byref(prob), B, Xb.data_ptr(), ws.data_ptr(),
                                            G.data_ptr(), 1, gx.data_ptr(), s), "bwd")
    return run


# B = 1: the single-graph apply (2-D X), the batched C ABI at B = 1 takes the same route
Xg = (Xb[0] if B == 1 else Xb).clone().requires_grad_(True)
Ya, Ga = (Yb[0], G[0]) if B == 1 else (Yb, G)


def apply():
    U_ = GLL.LaplaceLearningSparseHard.apply(Xg, Ya, 0.07, 1.0, k)
    torch.autograd.grad(U_, Xg, Ga)


def measure(label, fn, only_cg, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    qs = [cg] if only_cg else range(_lib.K_COUNT)
    for q in qs:
        _lib.prof_enable(q, 1)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    parts = []
    for q in qs:
        ms, cnt = _lib.prof_read(q)
        _lib.prof_enable(q, 0)
        if cnt:
            parts.append(f"{names[q].replace('_kernel', '')}={1e3 * ms / cnt:.2f}")
    print(f"{cfg} B={B} {label:13s} wall {1e6 * wall:8.1f} us | {' '.join(parts)}", flush=True)


for rnd in range(2):
    measure("abi", abi(False), False)
    measure("abi_cgonly", abi(False), True)
    measure("abi_fresh", abi(True), False)
    measure("apply", apply, False)
    measure("apply_cgonly", apply, True)
