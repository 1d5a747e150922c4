"""A/B of gll_problem.flags variants through the raw C ABI (diagnostic, run on the GPU box).

    python tools/ab_flags.py [--flags 0,4] [--configs ns,stress] [--batch 1,64] [--lib PATH]

For each config x batch x flags: mean launch time of every kernel (HIP events around each
launch), wall time per fwd+bwd with nothing else on the host path, CG iterations, and the
largest relative difference of U / gradX against the first flags value.
"""
import argparse
import ctypes as ct
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

EPS = {"plumbing": 1.0, "ns": 1.0, "fullysup": 1.0, "stress": "auto"}
ap = argparse.ArgumentParser()
ap.add_argument("--flags", default="0")
ap.add_argument("--configs", default="ns")
ap.add_argument("--batch", default="1,64")
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--lib", default="", help="another build of libgll.so to load instead (A/B of builds)")
ap.add_argument("--knob", type=int, default=-1, help="include/gll.h GLL_KNOB_* id to sweep")
ap.add_argument("--sink", action="store_true", help="pass a status sink (as the torch apply does)")
ap.add_argument("--values", default="0", help="values of --knob to sweep (0 = automatic)")
a = ap.parse_args()

if a.lib:
    _lib._lib = _lib._declare(ct.CDLL(os.path.abspath(a.lib)))
lib = _lib.lib()
names = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)]
s = torch.cuda.current_stream().cuda_stream
for cfg in a.configs.split(","):
    c = CONFIGS[cfg]
    n, m = c["base"] + c["batch"], c["batch"]
    for B in [int(b) for b in a.batch.split(",")]:
        Xs, Ys = [], []
        for g in range(min(B, 8)):
            X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=g)
            Xs.append(X_np)
            Ys.append(one_hot(lab[: c["base"]]))
        reps = (B + len(Xs) - 1) // len(Xs)
        X = torch.from_numpy(np.concatenate([np.stack(Xs)] * reps)[:B]).cuda().contiguous()
        Y = torch.from_numpy(np.concatenate([np.stack(Ys)] * reps)[:B]).cuda().contiguous()
        G = torch.from_numpy(np.stack([seeded_gbar(m, 10, 7 + g) for g in range(B)])).cuda()
        ref = None
        variants = [(int(f), int(gm)) for gm in a.values.split(",") for f in a.flags.split(",")]
        for flags, geom in variants:
            if a.knob >= 0:
                _lib.set_knob(a.knob, geom)
            prob = GLL.make_problem(n, c["d"], c["base"], 10, c["k"], 0.07, EPS[cfg], flags=flags)
            if a.sink:
                sink = torch.zeros(_lib.ST_NWORDS, dtype=torch.int32, device="cuda")
                prob.status_sink = sink.data_ptr()
            nb = lib.gll_workspace_bytes(ct.byref(prob))
            ws = torch.zeros(nb * B, dtype=torch.uint8, device="cuda")
            U = torch.empty(B, m, 10, dtype=torch.float64, device="cuda")
            gx = torch.empty(B, n, c["d"], dtype=torch.float32, device="cuda")

            def run():
                _lib.check(lib.gll_forward_batched(ct.byref(prob), B, X.data_ptr(), Y.data_ptr(), 0,
                                                   ws.data_ptr(), U.data_ptr(), s), "fwd")
                _lib.check(lib.gll_backward_batched(ct.byref(prob), B, X.data_ptr(), ws.data_ptr(),
                                                    G.data_ptr(), 1, gx.data_ptr(), s), "bwd")
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                run()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / a.reps
            for q in range(_lib.K_COUNT):
                _lib.prof_enable(q, 1)
            for _ in range(a.reps):
                run()
            torch.cuda.synchronize()
            per = []
            for q in range(_lib.K_COUNT):
                ms, cnt = _lib.prof_read(q)
                _lib.prof_enable(q, 0)
                if cnt:
                    per.append(f"{names[q].replace('_kernel', '')}={1e3 * ms / cnt:.2f}")
            st = (sink if a.sink else ws[: 4 * _lib.ST_NWORDS].view(torch.int32)).cpu().tolist()
            out = (U.cpu().numpy(), gx.cpu().numpy())
            diff = ""
            if ref is None:
                ref = out
            else:
                eu = np.abs(out[0] - ref[0]).max() / np.abs(ref[0]).max()
                eg = np.abs(out[1] - ref[1]).max() / np.abs(ref[1]).max()
                diff = f" dU={eu:.1e} dg={eg:.1e}"
            print(f"{cfg} B={B} flags={flags} knob={geom}: wall {1e6 * wall:8.1f} us/call-batch "
                  f"({1e6 * wall / B:.2f} us/graph) iters {st[_lib.ST_FWD_ITERS]}/"
                  f"{st[_lib.ST_BWD_ITERS]} | {' '.join(per)}{diff}", flush=True)
