"""Where the fused backward's last gradient waves spend their time (diagnostic, GPU box).

Loads the timestamp build (tools/libgll_trace.so.trace, a copy of _obj/libgll_trace.so made by
`python -m graphlearninglayer_amd.build --trace`), runs NS forward + backward through the C
ABI and reads, per gradient wave (one row each) of cg_grad_fused_kernel, the s_memrealtime
(100 MHz) stamps of: release seen, w loaded (+ first coefficients), products done, stored; plus
the row length and the wave's CU / XCC.  Prints the distribution of each phase after the
release and the slowest waves.
"""
import ctypes as ct
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from graphlearninglayer_amd import GLL  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

_tl = os.path.join(ROOT, "tools", "libgll_trace.so.trace")
lib = ct.CDLL(_tl if os.path.exists(_tl) else
              os.path.join(ROOT, "graphlearninglayer_amd", "_obj", "libgll_trace.so"))
lib.gll_workspace_bytes.restype = ct.c_size_t
lib.gll_trace_read_fz.argtypes = [ct.POINTER(ct.c_ulonglong)]
c = CONFIGS[os.environ.get("TRACE_CFG", "ns")]
n, base, d, k = c["base"] + c["batch"], c["base"], c["d"], c["k"]
dev = torch.device("cuda", 0)
X_np, lab = synth(base, n - base, d, r=c["r"], seed=0)
X = torch.from_numpy(X_np).to(dev)
Y = torch.from_numpy(one_hot(lab[:base])).to(dev)
g = torch.from_numpy(seeded_gbar(n - base, 10)).to(dev)
prob = GLL.make_problem(n, d, base, 10, k, 0.07, 1.0)
ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device=dev)
U = torch.empty(n - base, 10, dtype=torch.float64, device=dev)
gx = torch.empty(n, d, dtype=torch.float32, device=dev)
s = ct.c_void_p(torch.cuda.current_stream().cuda_stream)
vp = ct.c_void_p


def fwd():
    assert lib.gll_forward(ct.byref(prob), vp(X.data_ptr()), vp(Y.data_ptr()), 0,
                           vp(ws.data_ptr()), vp(U.data_ptr()), s) == 0


def bwd():
    assert lib.gll_backward(ct.byref(prob), vp(X.data_ptr()), vp(Y.data_ptr()), 0,
                            vp(ws.data_ptr()), vp(g.data_ptr()), 1, vp(gx.data_ptr()), s) == 0


for _ in range(20):
    fwd()
    bwd()
torch.cuda.synchronize()
rows_all = []
for rep in range(5):
    fwd()
    bwd()
    torch.cuda.synchronize()
    buf = (ct.c_ulonglong * (5 * 4096))()
    lib.gll_trace_read_fz(buf)
    a = np.array(buf[:], dtype=np.uint64).reshape(5, 4096)[:, :n].astype(np.int64)
    rel, wld, fma, sto, info = a
    t0 = rel.min()
    L = info & 0xFFFF
    cu = (info >> 16) & 0xFFFF
    xcc = (info >> 40) & 0xFF
    ph = {"release seen": rel - t0, "w loaded": wld - t0, "products done": fma - t0,
          "stored": sto - t0}
    print(f"--- rep {rep}: us after the first wave saw the release (n = {n} waves)")
    for nm, v in ph.items():
        q = np.percentile(v, [0, 50, 90, 99, 100]) * 0.01
        print(f"  {nm:14s} min {q[0]:5.2f} p50 {q[1]:5.2f} p90 {q[2]:5.2f} p99 {q[3]:5.2f} max {q[4]:5.2f}")
    dw = (wld - rel) * 0.01
    df = (fma - wld) * 0.01
    ds = (sto - fma) * 0.01
    print(f"  per wave: release->w {np.median(dw):.2f} (max {dw.max():.2f}), w->products "
          f"{np.median(df):.2f} (max {df.max():.2f}), products->stored {np.median(ds):.2f} "
          f"(max {ds.max():.2f})")
    slow = np.argsort(sto)[-8:]
    print("  slowest waves (row, len, xcc, cu, release, w, products, stored):")
    for i in slow[::-1]:
        print(f"    {i:5d} {L[i]:3d} {xcc[i]:2d} {cu[i]:5x} {0.01 * (rel[i] - t0):6.2f} "
              f"{0.01 * (wld[i] - t0):6.2f} {0.01 * (fma[i] - t0):6.2f} {0.01 * (sto[i] - t0):6.2f}")
    by_x = [0.01 * np.median(sto[xcc == x] - t0) for x in range(8) if np.any(xcc == x)]
    print("  median stored time by XCC: " + " ".join(f"{v:.2f}" for v in by_x))
    cor = np.corrcoef(L, sto)[0, 1]
    print(f"  corr(row length, stored time) {cor:.2f}; rows > 16 edges: {int((L > 16).sum())}")
    rows_all.append(sto - t0)
