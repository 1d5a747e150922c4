"""In-kernel timeline of one NS fwd+bwd call (diagnostic, GPU box).

Loads the timestamp build (_obj/libgll_trace.so, `python -m graphlearninglayer_amd.build
--trace`), runs forward then backward at the NS config through the C ABI and prints, per
kernel, first-workgroup entry -> last-workgroup exit, the gaps between consecutive kernels,
and the block-0 checkpoints of the CG kernel.  Clock: s_memrealtime, 100 MHz.
"""
import ctypes as ct
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

TICK_US = 0.01
# _obj/ stays on this side (.gpurunignore): copy the trace build next to this script to ship it
_tl = os.environ.get("TRACE_LIB", os.path.join(ROOT, "tools", "libgll_trace.so"))
lib = ct.CDLL(_tl if os.path.exists(_tl) else
              os.path.join(ROOT, "graphlearninglayer_amd", "_obj", "libgll_trace.so"))
lib.gll_workspace_bytes.restype = ct.c_size_t
lib.gll_trace_read.argtypes = [ct.c_int, ct.POINTER(ct.c_ulonglong)]
UNITS = {0: ("knn", ["gram", "select", "gram_wide", "gram48", "gram_bf3"]), 1: ("rows", ["row_build"]),
         2: ("solve", ["cg_ell", "cg_lds", "cg_csr"]), 3: ("grad", ["edge_coef", "grad_spmm"])}
CG_PTS = ["entry", "ell loaded+P", "ovf compacted", "rz/bb reduced", "it1 spmv", "it1 pAp",
          "it1 rr", "it1 P published", "loop done", "stored"]

cfg_name = os.environ.get("TRACE_CFG", "ns")
c = CONFIGS[cfg_name]
n, base, d, k = c["base"] + c["batch"], c["base"], c["d"], c["k"]
eps = float(os.environ.get("TRACE_EPS", "1.0"))
dev = torch.device("cuda", 0)
B = int(os.environ.get("TRACE_B", "1"))   # > 1: the batched entry points, B copies of the graph
X_np, lab = synth(base, n - base, d, r=c["r"], seed=0)
X = torch.from_numpy(np.stack([X_np] * B)).to(dev)
Y = torch.from_numpy(np.stack([one_hot(lab[:base])] * B)).to(dev)
g = torch.from_numpy(np.stack([seeded_gbar(n - base, 10)] * B)).to(dev)
prob = GLL.make_problem(n, d, base, 10, k, 0.07, eps, flags=int(os.environ.get("TRACE_FLAGS", "0")))
ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)) * B, dtype=torch.uint8, device=dev)
U = torch.empty(B, n - base, 10, dtype=torch.float64, device=dev)
gx = torch.empty(B, n, d, dtype=torch.float32, device=dev)
s = ct.c_void_p(torch.cuda.current_stream().cuda_stream)
vp = ct.c_void_p


def fwd():
    assert lib.gll_forward_batched(ct.byref(prob), B, vp(X.data_ptr()), vp(Y.data_ptr()), 0,
                                   vp(ws.data_ptr()), vp(U.data_ptr()), s) == 0


def bwd():
    assert lib.gll_backward_batched(ct.byref(prob), B, vp(X.data_ptr()), vp(ws.data_ptr()),
                                    vp(g.data_ptr()), 1, vp(gx.data_ptr()), s) == 0


def read_all():
    out = {}
    for u in UNITS:
        buf = (ct.c_ulonglong * 64)()
        lib.gll_trace_read(u, buf)
        out[u] = np.array(buf[:], dtype=np.uint64)
    return out


def timeline(tr, label):
    spans = []
    for u, (_, kns) in UNITS.items():
        for i, kn in enumerate(kns):
            a, b = int(tr[u][32 + 2 * i]), int(tr[u][33 + 2 * i])
            if a != 2 ** 64 - 1 and b != 0:
                spans.append((a, b, kn))
    spans.sort()
    t0 = spans[0][0]
    print(f"--- {label} (us from first entry)")
    prev = None
    for a, b, kn in spans:
        gap = "" if prev is None else f"  gap {TICK_US * (a - prev):6.2f}"
        print(f"{kn:10s} {TICK_US * (a - t0):7.2f} -> {TICK_US * (b - t0):7.2f}  "
              f"({TICK_US * (b - a):6.2f}){gap}")
        prev = b
    for u, (_, kns) in UNITS.items():
        for i, kn in enumerate(kns):
            last = int(tr[u][24 + i])
            if last:
                print(f"  {kn}: last workgroup entered at +{TICK_US * (last - int(tr[u][32 + 2 * i])):.2f}")
    g = tr[0].astype(np.int64)
    if g[10]:
        print("gram block 0: " + ", ".join(f"{nm} +{TICK_US * (g[q] - g[10]):.2f}" for q, nm in
                                          [(15, "chunk0 in LDS"), (11, "mfma done"), (12, "loop exit"),
                                           (13, "tile staged"), (14, "stored")] if g[q]))
    if g[21] and g[22] and g[14] > g[10]:
        mhz = (g[22] - g[21]) / ((g[14] - g[10]) / 100.0)
        print(f"gram block 0: shader clock {mhz:.0f} MHz (s_memtime / s_memrealtime)")
    if g[16] and g[20]:
        print("select wave 0: " + ", ".join(f"{nm} +{TICK_US * (g[q] - g[20]):.2f}" for q, nm in
                                           [(23, "row loaded"), (16, "scanned"), (17, "merged"), (18, "refined"),
                                            (19, "ranked+written")] if g[q]))
    rw = tr[1].astype(np.int64)
    rl = ["lists loaded", "staged (rev+ovf)", "sorted", "weights+deg", "ell/vr written", "rhs", "end"]
    for o, nm in ((0, "row_build row base"), (10, "row_build hub row")):
        if rw[o]:
            print(f"{nm}: " + ", ".join(f"{rl[q - 1]} +{TICK_US * (rw[o + q] - rw[o]):.2f}"
                                          for q in range(1, 8) if rw[o + q]) +
                  "".join(f", {lb} +{TICK_US * (rw[o + q] - rw[o]):.2f}"
                          for q, lb in ((8, "[overflow count read]"), (9, "[reverse list staged]")) if rw[o + q]))
    if rw[22]:
        print(f"row_build hub row: overflow list {rw[22]} entries, first batch matched "
              f"+{TICK_US * (rw[23] - rw[10]):.2f}")
    if rw[20] or rw[21]:
        print(f"row_build longest wave: every 16th row {TICK_US * rw[20]:.2f} us, hub rows {TICK_US * rw[21]:.2f} us")
    cyc = tr[2][10:16].astype(np.int64)
    if cyc[0] and cyc[5]:
        lab = ["update+store", "publish barrier", "spmv+dots", "reduce (dpp+lds+barrier)", "alpha/beta+p,s"]
        print("cg block 0 wave 0, iteration 3 (shader cycles): " +
              ", ".join(f"{lab[q]} {cyc[q + 1] - cyc[q]}" for q in range(5)) +
              f" | total {cyc[5] - cyc[0]}")
    fz = tr[2].astype(np.int64)
    if fz[16] and fz[32] and fz[32] < 2 ** 62:
        base = fz[32]   # first entry of the solve kernel (the CG role of the fused backward)
        print("fused backward (us from the first CG entry): " + ", ".join(
            f"{nm} +{TICK_US * (fz[q] - base):.2f}" for q, nm in
            [(16, "grad block C prefetch issued"), (17, "its wait over"), (18, "its rows stored"),
             (33, "last CG exit"), (19, "last grad exit")] if fz[q]))
    pts = tr[2][:10].astype(np.int64)
    if pts[0]:
        print("cg block 0: " + ", ".join(f"{CG_PTS[i]} +{TICK_US * (pts[i] - pts[0]):.2f}"
                                         for i in range(1, 10) if pts[i]))


for _ in range(10):
    fwd()
    bwd()
torch.cuda.synchronize()
for rep in range(3):
    for u in UNITS:
        lib.gll_trace_reset(u)
    fwd()
    torch.cuda.synchronize()
    timeline(read_all(), f"forward rep {rep}")
    for u in UNITS:
        lib.gll_trace_reset(u)
    bwd()
    torch.cuda.synchronize()
    timeline(read_all(), f"backward rep {rep}")
