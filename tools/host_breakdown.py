"""Host-side cost of one GLL step, piece by piece (diagnostic, run on the GPU box).

The NS step is host-bound when the GPU idles between steps (rocprof trace: ~25 us idle per
step).  This times, per step, the enqueue cost and the wall time of:
  raw C-ABI   gll_forward + gll_backward through ctypes, no torch autograd
  ext fwd     the C++ autograd node's forward only (no graph kept)
  step        apply + autograd.grad (the bench step)
  step/bwd()  apply + U.backward(g)
  torch op    a trivial torch kernel launch (x.add_(1)), for scale
  autograd    autograd.grad through a trivial GPU op (engine + device-thread hand-off)
"""
import ctypes as ct
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

c = CONFIGS["ns"]
dev = torch.device("cuda", 0)
X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
X = torch.from_numpy(X_np).to(dev).requires_grad_(True)
Y = torch.from_numpy(one_hot(lab[: c["base"]])).to(dev)
g = torch.from_numpy(seeded_gbar(c["batch"], 10)).to(dev)
lap = GLL.LaplaceLearningSparseHard.apply
N = 400


def timeit(label, fn, n=N):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(n):
        fn()
    e = time.perf_counter() - a
    torch.cuda.synchronize()
    w = time.perf_counter() - a
    print(f"{label:34s} enqueue {1e6 * e / n:8.1f} us   wall {1e6 * w / n:8.1f} us", flush=True)


lib = _lib.lib()
prob = GLL.make_problem(1000, 512, 500, 10, 10, 0.07, 1.0)
nb = lib.gll_workspace_bytes(ct.byref(prob))
s = torch.cuda.current_stream().cuda_stream
Xd = X.detach()
ws = torch.empty(nb, dtype=torch.uint8, device=dev)
Ud = torch.empty(500, 10, dtype=torch.float64, device=dev)
gx = torch.empty(1000, 512, dtype=torch.float32, device=dev)


def raw():
    lib.gll_forward(ct.byref(prob), Xd.data_ptr(), Y.data_ptr(), 0, ws.data_ptr(), Ud.data_ptr(), s)
    lib.gll_backward(ct.byref(prob), Xd.data_ptr(), None, 0, ws.data_ptr(), g.data_ptr(),
                     _lib.GLL_DT_F64, gx.data_ptr(), s)


def raw_fwd():
    lib.gll_forward(ct.byref(prob), Xd.data_ptr(), Y.data_ptr(), 0, ws.data_ptr(), Ud.data_ptr(), s)


def ext_fwd():
    with torch.no_grad():
        lap(X, Y, 0.07, 1.0, 10)


def step():
    U = lap(X, Y, 0.07, 1.0, 10)
    torch.autograd.grad(U, X, g)


def step_bwd():
    U = lap(X, Y, 0.07, 1.0, 10)
    U.backward(g)


t = torch.zeros(16, device=dev)


def tiny():
    t.add_(1)


a = torch.randn(1000, 512, device=dev, requires_grad=True)
ga = torch.randn(1000, 512, device=dev)


def tiny_grad():
    y = a * 2
    torch.autograd.grad(y, a, ga)


timeit("raw C-ABI fwd+bwd (ctypes)", raw)
timeit("raw C-ABI fwd (ctypes)", raw_fwd)
timeit("ext fwd (no_grad)", ext_fwd)
timeit("step: apply + autograd.grad", step)
timeit("step: apply + U.backward", step_bwd)
timeit("torch op x.add_(1)", tiny)
timeit("autograd.grad(a*2)", tiny_grad)
with torch.autograd.set_multithreading_enabled(False):
    timeit("step, autograd single-threaded", step)
    timeit("autograd.grad(a*2), single-threaded", tiny_grad)


def launch_only():   # one trivial HIP kernel through the C ABI's cheapest entry (status probe)
    lib.gll_backward(ct.byref(prob), Xd.data_ptr(), None, 0, ws.data_ptr(), g.data_ptr(),
                     _lib.GLL_DT_F64, gx.data_ptr(), s)


timeit("raw C-ABI bwd (2 launches)", launch_only)
