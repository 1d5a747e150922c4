"""Forward time of one large single graph with the pre-split Gram (default for d > 128) and the
inline 128-tile Gram (GLL_FLAG_GRAM_INLINE), at sizes past the stress shape (diagnostic, GPU box):
decides whether the single-graph routing in knn.hip launch_gram needs an n bound as well."""
import ctypes as ct
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import one_hot, synth  # noqa: E402

lib = _lib.lib()
for nu, d in [(20000, 256), (30000, 512), (30000, 1024)]:
    base = 250
    X, lab = synth(base, nu, d, r=1.0, seed=2)
    Xd = torch.from_numpy(X).cuda()
    Yd = torch.from_numpy(one_hot(lab[:base])).cuda()
    n = base + nu
    for name, flags in [("pre-split", 0), ("inline", _lib.FLAG_GRAM_INLINE)]:
        prob = GLL.make_problem(n, d, base, 10, 10, 0.07, 1.0, flags=flags)
        ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device="cuda")
        U = torch.empty(nu, 10, dtype=torch.float64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _lib.check(lib.gll_forward(ct.byref(prob), Xd.data_ptr(), Yd.data_ptr(),
                                       _lib.GLL_DT_F32, ws.data_ptr(), U.data_ptr(), s), "fwd")
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"n={n} d={d} {name:9s}: forward {1e3 * min(ts):8.2f} ms", flush=True)
        del ws
        torch.cuda.empty_cache()
