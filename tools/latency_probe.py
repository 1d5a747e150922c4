"""Fixed vs incremental cost of the latency-bound kernels at NS size (diagnostic, GPU box).

* CG: forward solve with max_iter = 1..12 (rtol 1e-30 so every column runs max_iter), timed
  with HIP events per launch -> slope = one PCG iteration, intercept = setup + launch.
* Gram / select / rows: n = 1000, d swept -> slope = one depth chunk of the MFMA pipeline.
"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import one_hot, synth  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.lib()
names = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)]


def timed_forward(n, base, d, k, max_iter=0, rtol=0.0, reps=30):
    X_np, lab = synth(base, n - base, d, r=1.0, seed=0)
    X = torch.from_numpy(X_np).to(dev)
    Y = torch.from_numpy(one_hot(lab[:base])).to(dev)
    prob = GLL.make_problem(n, d, base, 10, k, 0.07, 1.0)
    prob.max_iter = max_iter
    prob.rtol = rtol
    ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device=dev)
    U = torch.empty(n - base, 10, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def run():
        _lib.check(lib.gll_forward(ct.byref(prob), X.data_ptr(), Y.data_ptr(), 0, ws.data_ptr(),
                                   U.data_ptr(), s), "gll_forward")
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    for q in range(_lib.K_COUNT):
        _lib.prof_enable(q, 1)
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    out = {}
    for q in range(_lib.K_COUNT):
        ms, cnt = _lib.prof_read(q)
        _lib.prof_enable(q, 0)
        if cnt:
            out[names[q]] = 1e3 * ms / cnt
    st = ws[: 4 * _lib.ST_NWORDS].view(torch.int32).cpu().tolist()
    return out, st[_lib.ST_FWD_ITERS]


print("# CG forward, NS graph (n=1000, base=500, d=512, K=10), rtol=1e-30 -> fixed iterations")
for it in [1, 2, 3, 4, 6, 8, 12, 16]:
    t, iters = timed_forward(1000, 500, 512, 10, max_iter=it, rtol=1e-30)
    print(f"max_iter={it:3d} iters={iters:3d} cg_kernel={t['cg_kernel']:.2f} us", flush=True)
print("# graph build vs d (n=1000, K=10)")
for d in [16, 32, 64, 128, 256, 512, 1024]:
    t, _ = timed_forward(1000, 500, d, 10)
    print(f"d={d:5d} " + " ".join(f"{k}={v:.2f}" for k, v in t.items() if k != "cg_kernel"),
          flush=True)
