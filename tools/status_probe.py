"""kNN slow-path counters per call at the bench shapes (diagnostic, GPU box): rows that took the
exact candidate merge and rows whose candidate set failed the Gram-error certificate (exact
rescan).  A select launch lasts as long as its slowest row, so a handful of slow-path rows sets
the kernel's time at NS."""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, synth  # noqa: E402

for cfg, eps in [("ns", 1.0), ("fullysup", 1.0), ("ns", "auto")]:
    c = CONFIGS[cfg]
    for seed in range(3):
        X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=seed)
        Xd = torch.from_numpy(X).cuda()
        Y = torch.from_numpy(one_hot(lab[: c["base"]])).cuda()
        n, d = X.shape
        prob = GLL.make_problem(n, d, c["base"], 10, c["k"], 0.07, eps)
        lib = _lib.lib()
        ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device="cuda")
        U = torch.empty(n - c["base"], 10, dtype=torch.float64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        _lib.check(lib.gll_forward(ct.byref(prob), Xd.data_ptr(), Y.data_ptr(), _lib.GLL_DT_F32,
                                   ws.data_ptr(), U.data_ptr(), s), "gll_forward")
        st = ws[: 4 * _lib.ST_NWORDS].view(torch.int32).cpu().tolist()
        print(f"{cfg} eps={eps} seed={seed}: merge rows {st[_lib.ST_KNN_MERGE]}, "
              f"rescan rows {st[_lib.ST_KNN_RESCAN]}, fwd CG iters {st[_lib.ST_FWD_ITERS]}",
              flush=True)
