"""Where does a GLL step's wall time go on the host?  (diagnostic, run on the GPU box)

Times the Python/launch side of one fwd+bwd step with and without a device sync, and the
enqueue time of each piece, at the NS config.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

c = CONFIGS["ns"]
dev = torch.device("cuda", 0)
X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
X = torch.from_numpy(X_np).to(dev).requires_grad_(True)
Y = torch.from_numpy(one_hot(lab[: c["base"]])).to(dev)
g = torch.from_numpy(seeded_gbar(c["batch"], 10)).to(dev)
lap = GLL.LaplaceLearningSparseHard.apply
for _ in range(20):
    U = lap(X, Y, 0.07, 1.0, 10)
    torch.autograd.grad(U, X, g)
torch.cuda.synchronize()

N = 300
t_fwd = t_bwd = 0.0
t0 = time.perf_counter()
for _ in range(N):
    a = time.perf_counter()
    U = lap(X, Y, 0.07, 1.0, 10)
    b = time.perf_counter()
    torch.autograd.grad(U, X, g)
    t_fwd += b - a
    t_bwd += time.perf_counter() - b
t_enq = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"enqueue per step {1e6 * t_enq / N:.1f} us (fwd {1e6 * t_fwd / N:.1f}, bwd {1e6 * t_bwd / N:.1f}); "
      f"wall per step {1e6 * t_all / N:.1f} us")

# pieces of the forward in isolation
import ctypes as ct  # noqa: E402
from graphlearninglayer_amd import _lib  # noqa: E402

prob = GLL.make_problem(1000, 512, 500, 10, 10, 0.07, 1.0)
nb = _lib.lib().gll_workspace_bytes(ct.byref(prob))
s = torch.cuda.current_stream().cuda_stream
Xd = X.detach()
ws = torch.empty(nb, dtype=torch.uint8, device=dev)
Ud = torch.empty(500, 10, dtype=torch.float64, device=dev)
torch.cuda.synchronize()
for label, fn in [
    ("torch.empty ws+U", lambda: (torch.empty(nb, dtype=torch.uint8, device=dev),
                                  torch.empty(500, 10, dtype=torch.float64, device=dev))),
    ("gll_forward (C ABI only)", lambda: _lib.lib().gll_forward(ct.byref(prob), Xd.data_ptr(), Y.data_ptr(), 0,
                                                               ws.data_ptr(), Ud.data_ptr(), s)),
    ("current_stream()", lambda: torch.cuda.current_stream(dev).cuda_stream),
    ("X.detach().to().contiguous()", lambda: X.detach().to(device=dev, dtype=torch.float32).contiguous()),
]:
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(N):
        fn()
    e = time.perf_counter() - a
    torch.cuda.synchronize()
    w = time.perf_counter() - a
    print(f"{label:32s} enqueue {1e6 * e / N:8.1f} us   wall {1e6 * w / N:8.1f} us")
