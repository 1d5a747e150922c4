"""A/B of the whole-GPU CG variants (gridcg.hip; diagnostic, run on the GPU box).

    python tools/gridcg_probe.py [--variants classic,gv,gv_flat,gv_g128,gv_g64] [--laplace]

Variants are environment settings the library reads per call: GLL_GRID_CLASSIC (the round-2
two-barrier kernel), GLL_GRID_HIER (two-level barrier), GLL_GRID_G (workgroups).  For the
stress config (fwd+bwd through the C ABI): CG launch time from events in the dispatch packet,
iterations, and U / gradX differences against the first variant; with --laplace also the
utils.laplace solve at 60,250 points.
"""
import argparse
import ctypes as ct
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib, utils  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

VARIANTS = {
    "classic": {"GLL_GRID_CLASSIC": "1"},
    "gv": {},
    "gv_flat": {"GLL_GRID_HIER": "0"},
    "gv_g128": {"GLL_GRID_G": "128"},
    "gv_g64": {"GLL_GRID_G": "64"},
    "gv_g192": {"GLL_GRID_G": "192"},
    "gv_nt256": {"GLL_GRID_NT": "256"},
    "gv_nt1024": {"GLL_GRID_NT": "1024"},
    "gv_nt1024_g64": {"GLL_GRID_NT": "1024", "GLL_GRID_G": "64"},
    "gv_nt1024_g128": {"GLL_GRID_NT": "1024", "GLL_GRID_G": "128"},
    "mode_pipe": {"GLL_GRID_MODE": "0"},
    "mode_cg": {"GLL_GRID_MODE": "1"},
}
KEYS = ("GLL_GRID_CLASSIC", "GLL_GRID_HIER", "GLL_GRID_G", "GLL_GRID_NT", "GLL_GRID_MODE")

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="classic,gv,gv_flat,gv_g128,gv_g64")
ap.add_argument("--configs", default="stress")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--laplace", action="store_true")
ap.add_argument("--laplace-variants", default="")
a = ap.parse_args()


def set_variant(v):
    for k in KEYS:
        os.environ.pop(k, None)
    os.environ.update(VARIANTS[v])


lib = _lib.lib()
s = torch.cuda.current_stream().cuda_stream
kid = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)].index("cg_kernel")
for cfg in a.configs.split(","):
    c = CONFIGS[cfg]
    n, m = c["base"] + c["batch"], c["batch"]
    eps = "auto" if cfg == "stress" else 1.0
    X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
    X = torch.from_numpy(X_np).cuda()
    Y = torch.from_numpy(one_hot(lab[: c["base"]])).cuda()
    G = torch.from_numpy(seeded_gbar(m, 10, 7)).cuda()
    flags = _lib.FLAG_CG_GRID if m <= 2048 else 0
    prob = GLL.make_problem(n, c["d"], c["base"], 10, c["k"], 0.07, eps, flags=flags)
    ws = torch.zeros(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device="cuda")
    U = torch.empty(m, 10, dtype=torch.float64, device="cuda")
    gx = torch.empty(n, c["d"], dtype=torch.float32, device="cuda")

    def run():
        _lib.check(lib.gll_forward(ct.byref(prob), X.data_ptr(), Y.data_ptr(), 0, ws.data_ptr(),
                                   U.data_ptr(), s), "fwd")
        _lib.check(lib.gll_backward(ct.byref(prob), X.data_ptr(), None, 0, ws.data_ptr(),
                                    G.data_ptr(), 1, gx.data_ptr(), s), "bwd")

    ref = None
    for v in a.variants.split(","):
        set_variant(v)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            run()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.reps
        _lib.prof_enable(kid, 1)
        for _ in range(a.reps):
            run()
        torch.cuda.synchronize()
        ms, cnt = _lib.prof_read(kid)
        _lib.prof_enable(kid, 0)
        st = ws[: 4 * _lib.ST_NWORDS].view(torch.int32).cpu().tolist()
        out = (U.cpu().numpy(), gx.cpu().numpy())
        diff = ""
        if ref is None:
            ref = out
        else:
            eu = np.abs(out[0] - ref[0]).max() / np.abs(ref[0]).max()
            eg = np.abs(out[1] - ref[1]).max() / np.abs(ref[1]).max()
            diff = f" dU={eu:.1e} dg={eg:.1e}"
        fin = bool(np.isfinite(out[0]).all() and np.isfinite(out[1]).all())
        print(f"{cfg} {v:8s}: call {1e6 * wall:8.1f} us, CG {1e3 * ms / max(cnt, 1):7.1f} us/launch "
              f"(n={cnt}), iters {st[_lib.ST_FWD_ITERS]}/{st[_lib.ST_BWD_ITERS]} nonconv "
              f"{st[_lib.ST_FWD_NONCONV]}/{st[_lib.ST_BWD_NONCONV]} failed {st[_lib.ST_SOLVE_FAILED]}"
              f" finite {fin}{diff}", flush=True)
    del X, ws, gx
    torch.cuda.empty_cache()

if a.laplace:
    nl, nu, d = 250, 60000, 128
    X, labels = synth(nl, nu, d, C=10, r=1.0, seed=3)
    Xd = torch.from_numpy(X).cuda()
    utils.laplace(Xd[:4000], labels[:nl])
    ref = None
    orig = GLL.refined_solve
    rec = {}

    def timed_solve(*args, **kw):   # solve time, CG iterations and launches of one laplace call
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.prof_enable(kid, 1)
        out = orig(*args, **kw)
        torch.cuda.synchronize()
        ms, cnt = _lib.prof_read(kid)
        _lib.prof_enable(kid, 0)
        rec.update(solve_ms=1e3 * (time.perf_counter() - t0), iters=out[2], cg_ms=ms, launches=cnt)
        return out

    GLL.refined_solve = timed_solve
    utils.GLL.refined_solve = timed_solve
    for v in (a.laplace_variants or a.variants).split(","):
        set_variant(v)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            Ul = utils.laplace(Xd, labels[:nl], knn_num=50, epsilon=1.0, tau=1e-8)
            t = time.perf_counter() - t0
        acc = 100.0 * np.mean(Ul.argmax(1) == labels[nl:])
        diff = "" if ref is None else f" dU={np.abs(Ul - ref).max() / np.abs(ref).max():.1e}"
        ref = Ul if ref is None else ref
        it = max(rec.get("iters", 0), 1)
        print(f"laplace n={nl + nu} {v:8s}: {t * 1e3:.1f} ms (solve {rec.get('solve_ms', 0):.1f} ms: "
              f"{rec.get('launches', 0)} CG launches {rec.get('cg_ms', 0):.1f} ms, {it} iterations, "
              f"{1e3 * rec.get('cg_ms', 0) / it:.1f} us/iter), GL accuracy {acc:.2f}%{diff}",
              flush=True)
