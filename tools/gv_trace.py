"""Timeline of the whole-GPU CG's iteration 3 (cg_gv_kernel, gridcg.hip) at the stress config
(diagnostic, GPU box; the trace build copied to tools/libgll_trace.so).

Block 0's checkpoints (s_memrealtime, 100 MHz) and the spread of every workgroup's arrival at
and release from that iteration's grid barrier.
"""
import ctypes as ct
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from graphlearninglayer_amd import GLL  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, synth  # noqa: E402

TICK_US = 0.01
lib = ct.CDLL(os.path.join(ROOT, "tools", "libgll_trace.so"))
lib.gll_workspace_bytes.restype = ct.c_size_t
PTS = {11: "iteration start", 12: "partials published", 13: "barrier released",
       14: "partials loaded + SpMV", 15: "partials reduced", 16: "step sizes", 17: "updates done",
       18: "next iteration start"}
cfg = os.environ.get("TRACE_CFG", "stress")
c = CONFIGS[cfg]
n = c["base"] + c["batch"]
X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
X = torch.from_numpy(X_np).cuda()
Y = torch.from_numpy(one_hot(lab[: c["base"]])).cuda()
prob = GLL.make_problem(n, c["d"], c["base"], 10, c["k"], 0.07, "auto")
ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device="cuda")
U = torch.empty(c["batch"], 10, dtype=torch.float64, device="cuda")
s = ct.c_void_p(torch.cuda.current_stream().cuda_stream)
buf = (ct.c_ulonglong * 64)()
wg = (ct.c_ulonglong * (2 * 3 * 4096))()
for rep in range(4):
    lib.gll_trace_reset(4)
    assert lib.gll_forward(ct.byref(prob), ct.c_void_p(X.data_ptr()), ct.c_void_p(Y.data_ptr()),
                           0, ct.c_void_p(ws.data_ptr()), ct.c_void_p(U.data_ptr()), s) == 0
    torch.cuda.synchronize()
    lib.gll_trace_read(4, buf)
    lib.gll_trace_read_wg(4, wg)
    t = list(buf)
    t0 = t[11]
    if rep == 0 or not t0:
        continue
    print(f"--- rep {rep}: kernel {TICK_US * (t[35] - t[34]):.2f} us, iteration 3 (block 0, us from its start)")
    prev = t0
    for i in range(12, 19):
        print(f"  {PTS[i]:24s} {TICK_US * (t[i] - t0):7.2f}  (+{TICK_US * (t[i] - prev):.2f})")
        prev = t[i]
    a = np.array(wg[:4096], dtype=np.int64)
    r = np.array(wg[4096:8192], dtype=np.int64)
    live = a > 0
    a, r = a[live], r[live]
    print(f"  barrier: {live.sum()} workgroups; arrivals span {TICK_US * (a.max() - a.min()):.2f} us "
          f"(median at +{TICK_US * (np.median(a) - a.min()):.2f}), last arrival -> releases "
          f"{TICK_US * (r.min() - a.max()):.2f} .. {TICK_US * (r.max() - a.max()):.2f} us")
    print(f"  block 0 arrived at +{TICK_US * (a[0] - a.min()):.2f}; slowest 5 blocks: "
          f"{np.argsort(a)[-5:].tolist()}")
