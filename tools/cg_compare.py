"""CG kernel time: per-column workgroup kernels vs the grid-wide cooperative CG (diagnostic)."""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

lib = _lib.lib()
kid = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)].index("cg_kernel")
for cfg, eps in [("ns", 1.0), ("stress", "auto")]:
    c = CONFIGS[cfg]
    n = c["base"] + c["batch"]
    X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
    X = torch.from_numpy(X_np).cuda()
    Y = torch.from_numpy(one_hot(lab[: c["base"]])).cuda()
    g = torch.from_numpy(seeded_gbar(c["batch"], 10)).cuda()
    for flags in (0, _lib.FLAG_CG_GRID):
        prob = GLL.make_problem(n, c["d"], c["base"], 10, c["k"], 0.07, eps, flags=flags)
        ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device="cuda")
        U = torch.empty(c["batch"], 10, dtype=torch.float64, device="cuda")
        gx = torch.empty(n, c["d"], dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream

        def run():
            _lib.check(lib.gll_forward(ct.byref(prob), X.data_ptr(), Y.data_ptr(), 0, ws.data_ptr(),
                                       U.data_ptr(), s), "fwd")
            _lib.check(lib.gll_backward(ct.byref(prob), X.data_ptr(), None, 0, ws.data_ptr(),
                                        g.data_ptr(), 1, gx.data_ptr(), s), "bwd")
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        _lib.prof_enable(kid, 1)
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        ms, cnt = _lib.prof_read(kid)
        _lib.prof_enable(kid, 0)
        st = ws[: 4 * _lib.ST_NWORDS].view(torch.int32).cpu().tolist()
        print(f"{cfg:7s} flags={flags}: cg {1e3 * ms / cnt:8.1f} us/launch, iters fwd/bwd "
              f"{st[_lib.ST_FWD_ITERS]}/{st[_lib.ST_BWD_ITERS]}, U[0,:3]={U[0, :3].tolist()}",
              flush=True)
