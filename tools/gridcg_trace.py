"""Timeline of the grid-wide CG (block 0, iteration 1) at NS with GLL_FLAG_CG_GRID (trace build)."""
import ctypes as ct
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, synth  # noqa: E402

lib = ct.CDLL(os.path.join(ROOT, "graphlearninglayer_amd", "_obj", "libgll_trace.so"))
lib.gll_workspace_bytes.restype = ct.c_size_t
NAMES = {0: "setup+bar", 2: "A spmv", 3: "bar A", 4: "B update", 5: "bar B", 6: "it1 end",
         1: "loop done"}
for cfg, eps in [("ns", 1.0), ("stress", "auto")]:
    c = CONFIGS[cfg]
    n = c["base"] + c["batch"]
    X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
    X = torch.from_numpy(X_np).cuda()
    Y = torch.from_numpy(one_hot(lab[: c["base"]])).cuda()
    prob = GLL.make_problem(n, c["d"], c["base"], 10, c["k"], 0.07, eps, flags=_lib.FLAG_CG_GRID)
    ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device="cuda")
    U = torch.empty(c["batch"], 10, dtype=torch.float64, device="cuda")
    s = ct.c_void_p(torch.cuda.current_stream().cuda_stream)
    for rep in range(3):
        lib.gll_trace_reset(4)
        assert lib.gll_forward(ct.byref(prob), ct.c_void_p(X.data_ptr()), ct.c_void_p(Y.data_ptr()),
                               0, ct.c_void_p(ws.data_ptr()), ct.c_void_p(U.data_ptr()), s) == 0
        torch.cuda.synchronize()
        buf = (ct.c_ulonglong * 64)()
        lib.gll_trace_read(4, buf)
        t = np.array(buf[:], dtype=np.uint64).astype(np.int64)
        ent, ext = t[32], t[33]
        pts = {k: (t[k] - ent) / 100.0 for k in NAMES if t[k]}
        print(f"{cfg} rep {rep}: kernel {(ext - ent) / 100.0:.2f} us; " +
              ", ".join(f"{NAMES[k]} {v:.2f}" for k, v in sorted(pts.items(), key=lambda kv: kv[1])),
              flush=True)
