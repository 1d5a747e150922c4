"""Per-kernel time under gll_problem.flags variants (diagnostic A/B, GPU box).

FLAGS env: comma list of gll_problem.flags values to compare (default "0,2": wide 128-tile
Gram vs 64-tile Gram; "0,1": per-column vs whole-GPU CG)."""
import ctypes as ct
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

lib = _lib.lib()
names = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)]
flags_list = [int(f) for f in os.environ.get("FLAGS", "0,2").split(",")]
for cfg, eps, B in [("ns", 1.0, 1), ("ns", 1.0, 64), ("stress", "auto", 1)]:
    c = CONFIGS[cfg]
    n = c["base"] + c["batch"]
    Xs, Ys = [], []
    for g in range(min(B, 8)):
        X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=g)
        Xs.append(X)
        Ys.append(one_hot(lab[: c["base"]]))
    reps = (B + 7) // 8
    X = torch.from_numpy(np.concatenate([np.stack(Xs)] * reps)[:B]).cuda().contiguous()
    Y = torch.from_numpy(np.concatenate([np.stack(Ys)] * reps)[:B]).cuda().contiguous()
    G = torch.from_numpy(np.stack([seeded_gbar(c["batch"], 10, g) for g in range(B)])).cuda()
    for flags in flags_list:
        prob = GLL.make_problem(n, c["d"], c["base"], 10, c["k"], 0.07, eps, flags=flags)
        ws = torch.empty(B * lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8,
                         device="cuda")
        U = torch.empty(B, c["batch"], 10, dtype=torch.float64, device="cuda")
        gx = torch.empty(B, n, c["d"], dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream

        def run():
            _lib.check(lib.gll_forward_batched(ct.byref(prob), B, X.data_ptr(), Y.data_ptr(), 0,
                                               ws.data_ptr(), U.data_ptr(), s), "fwd")
            _lib.check(lib.gll_backward_batched(ct.byref(prob), B, X.data_ptr(), ws.data_ptr(),
                                                G.data_ptr(), 1, gx.data_ptr(), s), "bwd")
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        for q in range(_lib.K_COUNT):
            _lib.prof_enable(q, 1)
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        parts = []
        for q in range(_lib.K_COUNT):
            ms, cnt = _lib.prof_read(q)
            _lib.prof_enable(q, 0)
            if cnt:
                parts.append(f"{names[q]}={1e3 * ms / cnt:.1f}")
        print(f"{cfg} B={B} flags={flags}: " + " ".join(parts), flush=True)
