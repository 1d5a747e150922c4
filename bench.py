"""GLL fwd+bwd throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config ns|fullysup|stress|plumbing]
    torchrun --nproc-per-node N bench.py --gpus N ...        (one process per GPU)

`--gpus N` with N > 1 and no WORLD_SIZE in the environment starts the N ranks itself: it runs
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...` as a child
process before anything touches the GPU and exits with the child's status (rank 0's JSON
line is the child's stdout).  Under an outer launcher WORLD_SIZE must equal N.
`--dry-run` replaces the GPU leg by a CPU stand-in step over gloo, so the launcher, the
coalesced prediction gather and the max-over-ranks timing can be tested on a CPU box.

One step = one `LaplaceLearningSparseHard.apply` forward (kNN graph built from scratch)
+ the backward of a fixed seeded upstream gradient dL/dU, on the rank's own synthetic
minibatch graph (seed = rank; SURVEY.md §8d generator), plus the asynchronous RCCL
all_gather of the predictions U that the sharded path performs (§8e), coalesced over
GATHER_EVERY calls.  Inputs are resident
in HBM before timing starts.  Rank 0 prints ONE JSON line; `value` = calls/s over all ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.parallel import (PredictionGatherer, distinct_devices,  # noqa: E402
                                              rank_identity, shard_rank_seed)
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402

METRIC = "GLL fwd+bwd calls/sec (base=500,batch=500,d=512,k=10) at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
MFMA_F32_PEAK_TFS = 157.3    # dense fp32 MFMA (v_mfma_f32_32x32x2_f32), spec
MFMA_BF16_PEAK_TFS = 2500.0  # dense bf16 MFMA, spec (~2.5 PF; 2:1-sparse figures never used)
# The Gram runs split-bf16 (x = hi + lo, three bf16 products per fp32 product) over the upper
# triangle of tiles: ~1.5 executed bf16 MFMA flops per algorithmic flop 2n^2 d, so its MFMA
# roof in algorithmic flops is the bf16 peak / 1.5.
GRAM_ROOF_TFS = MFMA_BF16_PEAK_TFS / 1.5
PROF_PERIOD = 7              # event-bracket every 7th launch of the dominant kernel (odd: the
                             # CG runs twice per step, so both the forward and adjoint get sampled)
GATHER_EVERY = 8             # calls per coalesced all_gather of the predictions
EPS = {"plumbing": 1.0, "ns": 1.0, "fullysup": 1.0, "stress": "auto"}
TAU = {"plumbing": 0.07, "ns": 0.07, "fullysup": 0.07, "stress": 0.07}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget of the CPU-baseline sample (rank 0, N=1 only); 0 disables")
    ap.add_argument("--no-profile", action="store_true", help="skip kernel event timing")
    ap.add_argument("--batch", type=int, default=64,
                    help="graphs per launch of the batched entry point measured beside the "
                         "headline (SURVEY.md §8f-2); 0 disables")
    ap.add_argument("--share-gpu", action="store_true",
                    help="diagnostic: every rank on cuda:0 over gloo (RCCL refuses two ranks on "
                         "one GPU), to run the real multi-rank GPU leg on a one-GPU box; the "
                         "JSON line is marked and is no scaling measurement")
    ap.add_argument("--autograd-thread", default="auto", choices=["auto", "caller", "device"],
                    help="where torch's autograd engine runs the backward: 'caller' = the calling "
                         "thread (torch.autograd.set_multithreading_enabled(False)), 'device' = "
                         "the engine's per-device worker thread (torch's default), 'auto' = "
                         "whichever ran a short untimed probe of each faster on this host; the "
                         "other mode is measured too and reported as `autograd_other_thread`")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU stand-in step over gloo instead of the GPU path (launcher and "
                         "gather test; the JSON line is marked dry_run and is no measurement)")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(a) -> int:
    """Start `a.gpus` ranks of this script under torch.distributed.run (one process per GPU,
    RCCL over xGMI) and return the launcher's exit status.  Runs before any GPU call: this
    process only waits for its child."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host driver
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def cg_spmvs(iters, B, m, n, K, C=10):
    """Matrix passes (SpMVs) of one CG solve of `iters` iterations, by the form the library's
    dispatch takes (solve.hip cg_dispatch, in its order): the whole-GPU CG for a single graph
    past m = 2048 and the balanced kernel where row_build packs virtual rows
    (gll_internal.h vr_threads: U-block rows longer than 12 entries) make one pass per
    iteration plus the pre-step; so do the batched 2- and 4-row register-ELL geometries.  The
    register-ELL kernel runs the Neumann-preconditioned form -- two passes per iteration plus
    two in setup -- wherever a thread owns one row: m <= 256, m <= 512 for a single graph or at
    most 256 column workgroups (B x C), 512 < m <= 1024."""
    if B == 1 and C <= 16 and m > 2048:
        return iters + 1
    vr_len = 1.4 * (K - 1) * m / n
    if m <= 2048 and vr_len > 12.0 and -(-m * (vr_len / 8 + 0.5) // 512) <= 10:
        return iters + 1
    one_row = m <= 256 or (m <= 512 and (B == 1 or B * C <= 256)) or 512 < m <= 1024
    return 2 * iters + 2 if one_row else iters + 1


def kernel_units(cfg, graph_stats, iters_fwd, iters_bwd, auto_eps, B=1):
    """Algorithmic work per launch of each kernel (SURVEY.md §8d byte/flop model)."""
    n, d, K, m, C = cfg["n"], cfg["d"], cfg["k"], cfg["batch"], 10
    E, nnz_uu = graph_stats
    b_spmv = 8 * nnz_uu + 8 * m + 8 * m * C
    u = {
        "gram_d2_kernel": ("mfma", 2.0 * n * n * d),
        "knn_select_kernel": ("hbm", 4.0 * n * n + 8.0 * n * K),
        "row_build_kernel": ("hbm", 16.0 * E + 8.0 * n * K + 4 * n + 4 * m * C),
        # SURVEY §8d SpMV roofline: B_spmv per matrix pass (the matrix and one gathered
        # vector), times the passes the solve made; the call roofline prices a whole CG
        # iteration instead (cg_iteration_bytes)
        "cg_kernel": ("hbm", 0.5 * (cg_spmvs(iters_fwd, B, m, n, K) + cg_spmvs(iters_bwd, B, m, n, K))
                      * b_spmv),
        "edge_coef_kernel": ("hbm", 16.0 * E + 8.0 * n * C),
        "grad_spmm_kernel": ("hbm", (12.0 * E + 8.0 * n * d) if auto_eps
                             else (8.0 * E + 8.0 * n * C + 8.0 * n * d)),
    }
    # the fused backward of a single small graph (adjoint CG + feature gradient, one launch)
    u["cg_grad_fused_kernel"] = ("hbm", cg_spmvs(iters_bwd, B, m, n, K) * b_spmv
                                 + u["grad_spmm_kernel"][1])
    return u


def cg_iteration_bytes(cfg, graph_stats, iters_fwd, iters_bwd, B=1):
    """§8d's whole CG iteration, B_spmv + 28 mC: the SpMV plus the vector updates (x, r, p, z
    read/written once each), which this library keeps in registers and LDS -- an 'effective'
    figure, reported beside the SpMV roofline and used by the call roofline.  Matrix passes
    as the solver makes them (cg_spmvs)."""
    m, C, n, K = cfg["batch"], 10, cfg["n"], cfg["k"]
    _, nnz_uu = graph_stats
    b_spmv = 8 * nnz_uu + 8 * m + 8 * m * C
    return 0.5 * sum(cg_spmvs(it, B, m, n, K) * b_spmv + it * 28 * m * C for it in (iters_fwd, iters_bwd))


def cg_roofline_extras(work_spmv, work_iter, avg_s, traffic):
    """Labelled companions of the SpMV roofline of one CG launch."""
    out = {"effective_incl_vector_bytes": {
        "work_per_launch": work_iter,
        "achieved_GBs": round(work_iter / avg_s / 1e9, 3),
        "frac": round(work_iter / avg_s / 1e9 / HBM_PEAK_GBS, 5),
        "note": "SURVEY §8d 'one CG iteration' bytes (B_spmv + 28 mC): counts the vector "
                "updates, which live in registers / LDS here, so this overstates HBM use"}}
    if traffic:
        out["pmc_traffic"] = {"bytes_per_launch": traffic,
                              "GBs": round(traffic / avg_s / 1e9, 3),
                              "frac": round(traffic / avg_s / 1e9 / HBM_PEAK_GBS, 5),
                              "note": "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch "
                                      "(committed PMC pass) over the live launch time"}
    return out


# C-ABI kernel ids (gll_kernel_name) -> device symbols as rocprofv3 names them.  The Gram id
# covers several launches on the pre-split route: gram_split_kernel (hi/lo planes),
# gram_pk2_kernel (the main 256-tile GEMM) and gram_pk_kernel (its 128-subtile tail); single
# small graphs run gram_bf3s_kernel (256 < d <= 512) or gram_bf3h_kernel (d <= 128) alone.
# The main kernel is listed first.
PMC_SYMBOLS = {"gram_d2_kernel": ["gram_pk2_kernel", "gram_bf3s_kernel", "gram_bf3w_kernel",
                                  "gram_bf3_kernel", "gram_bf3h_kernel", "gram_pk_kernel"],
               "knn_select_kernel": ["knn_select_kernel", "knn_select_wide_kernel"],
               "row_build_kernel": ["row_build_kernel"],
               "cg_kernel": ["cg_ell_kernel", "cg_vr_kernel", "cg_gv_kernel", "cg_grid_kernel",
                             "cg_lds_kernel"],
               "edge_coef_kernel": ["edge_coef_kernel"], "grad_spmm_kernel": ["grad_spmm_kernel", "grad_chunk_kernel"],
               "cg_grad_fused_kernel": ["cg_grad_fused_kernel"]}
# the Gram's launches by role, for the MFMA counters (reported separately)
GRAM_ROLES = (("main", "gram_pk2_kernel"), ("tail", "gram_pk_kernel"),
              ("single", "gram_bf3s_kernel"), ("inline", "gram_bf3w_kernel"),
              ("inline", "gram_bf3_kernel"), ("inline", "gram_bf3h_kernel"))


def build_profile_tags():
    """Profile-session tags recorded against THIS library build (profiles/<tag>_build.json,
    written by tools/prof_session.sh with the library's gll_build_id), newest first.  bench.py
    cites only these: a summary of another build is never cited, whatever its name."""
    import glob
    bid = _lib.build_id()
    tags = []
    for p in glob.glob(os.path.join(ROOT, "profiles", "*_build.json")):
        try:
            with open(p) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        if doc.get("build_id") == bid:
            tags.append((doc.get("recorded", ""), os.path.basename(p)[: -len("_build.json")]))
    return [t for _, t in sorted(tags, reverse=True)]


def _build_profile(name_of_tag):
    """profiles/<file> of the newest session of this build holding it, or None."""
    for tag in build_profile_tags():
        rel = os.path.join("profiles", name_of_tag(tag))
        if os.path.exists(os.path.join(ROOT, rel)):
            return rel
    return None


def pmc_traffic(config, kernel):
    """HBM-side bytes per launch of `kernel` from this build's PMC summary
    (profiles/<tag>_pmc_<config>.json, tools/pmc_summary.py over separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this same bench command), or None."""
    rel = _build_profile(lambda t: f"{t}_pmc_{config}.json")
    if rel is None:
        return None
    with open(os.path.join(ROOT, rel)) as f:
        doc = json.load(f)
    for sym in PMC_SYMBOLS.get(kernel, []):
        if sym in doc["kernels"]:
            return round(doc["kernels"][sym]["traffic_bytes"], 1)
    return None


def rocprof_stats(config):
    """This build's rocprofv3 --kernel-trace --stats summary of `config`, or None."""
    return _build_profile(lambda t: f"{t}_{config}_kernel_stats.csv")


def rocprof_avg_us(rel, kernel):
    """Mean rocprof duration (us) per C-ABI launch of `kernel` in a committed kernel_stats CSV:
    the summed durations of its device symbols over the calls of the first symbol present (the
    Gram id spans gram_split + the main GEMM + its tail; the events bracket that whole span)."""
    import csv
    if rel is None:
        return None
    tot_ns, calls = 0.0, {}
    syms = PMC_SYMBOLS[kernel] + (["gram_split_kernel"] if kernel == "gram_d2_kernel" else [])
    with open(os.path.join(ROOT, rel)) as f:
        for row in csv.DictReader(f):
            name = row["Name"]
            for sym in syms:
                if f"::{sym}<" in name or f"::{sym}(" in name:
                    tot_ns += float(row["TotalDurationNs"])
                    calls[sym] = calls.get(sym, 0) + int(row["Calls"])
                    break
    main = next((calls[sym] for sym in PMC_SYMBOLS[kernel] if sym in calls), 0)
    return round(tot_ns / main / 1e3, 3) if main else None


def gram_mfma_pmc(config):
    """The Gram's MFMA counters from this build's summary (profiles/<tag>_mfma_<config>.json,
    tools/mfma_summary.py over a rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16
    SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE pass), each Gram launch by role
    (main GEMM, tail, single-graph kernel), or None."""
    rel = _build_profile(lambda t: f"{t}_mfma_{config}.json")
    if rel is None:
        return None
    with open(os.path.join(ROOT, rel)) as f:
        doc = json.load(f)
    out = {}
    for role, sym in GRAM_ROLES:
        e = doc["kernels"].get(sym)
        if e and "exec_bf16_tflops" in e and role not in out:
            out[role] = {"kernel": sym, "exec_bf16_tflops": e["exec_bf16_tflops"],
                         "exec_frac_of_bf16_peak": e["exec_flops_frac_of_peak"],
                         "mfma_busy_frac": e.get("mfma_busy_frac"),
                         "duration_us": e["duration_us"]}
    if not out:
        return None
    out["source"] = rel
    return out


def batched_measure(c, eps, tau, k, B, gstats, dev, rank, steps=20, warmup=5):
    """B independent graphs of the workload per call of the batched entry point (X: B x n x d):
    whole-batch fwd+bwd throughput, and the CG kernel against the HBM roofline, where one
    launch now carries B graphs' SpMVs ('reported at batched NS')."""
    distinct = min(B, 8)   # a few distinct graphs, tiled: timing does not depend on content
    Xs, Ys = [], []
    for g in range(distinct):
        X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=1000 * rank + g)
        Xs.append(X)
        Ys.append(one_hot(lab[: c["base"]]))
    reps = (B + distinct - 1) // distinct
    Xb = torch.from_numpy(np.concatenate([np.stack(Xs)] * reps)[:B]).to(dev).requires_grad_(True)
    Yb = torch.from_numpy(np.concatenate([np.stack(Ys)] * reps)[:B]).to(dev)
    G = torch.from_numpy(np.stack([seeded_gbar(c["batch"], 10, 1234 + g) for g in range(B)])).to(dev)
    lap = GLL.LaplaceLearningSparseHard.apply

    def step():
        U = lap(Xb, Yb, tau, eps, k)
        return torch.autograd.grad(U, Xb, G)

    # the batched launches' own CG iterations (their solver differs from the single graph's)
    it_f, it_b = _cg_iters(Xb, Yb, tau, eps, k, G)
    units = kernel_units(c, gstats, it_f, it_b, isinstance(eps, str), B=B)
    cg_iter_work = cg_iteration_bytes(c, gstats, it_f, it_b, B=B)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    kid = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)].index("cg_kernel")
    # the batch throughput: a pass with no kernel events (they cost the step time, main())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the CG launch times: every launch of every kernel bracketed (a lone bracket on the CG reads
    # long: see main()) in a second pass; an untimed pass first fills the event pool, so the
    # measured one creates no event
    for q in range(_lib.K_COUNT):
        _lib.prof_enable(q, 1)
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    for q in range(_lib.K_COUNT):
        _lib.prof_read(q)
        _lib.prof_enable(q, 1)
    t1 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    elapsed_ev = time.perf_counter() - t1
    ms, cnt = _lib.prof_read(kid)
    for q in range(_lib.K_COUNT):
        _lib.prof_enable(q, 0)
        _lib.prof_read(q)
    bound, work = units["cg_kernel"]
    avg_s = ms / cnt / 1e3
    achieved = B * work / avg_s / 1e9
    traffic = pmc_traffic(f"{c['name']}_b{B}", "cg_kernel")
    roof = {"kernel": "cg_kernel", "bound": bound,
            "definition": "SURVEY §8d SpMV roofline: B_spmv x iterations x B graphs / CG launch "
                          "time / 8 TB/s, B_spmv = 8 nnz_off(Luu) + 8 m + 8 m C",
            "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "spmv_frac": round(achieved / HBM_PEAK_GBS, 5),
            "work_per_launch": B * work, "avg_launch_us": round(avg_s * 1e6, 3),
            "launches": cnt, "traffic": traffic,
            "rocprof_stats": rocprof_stats(f"{c['name']}_b{B}")}
    # the same SpMV roofline from this build's committed rocprofv3 summary (the profiler's
    # kernel durations read ~2 us longer than the dispatch-packet events per launch)
    rp_us = rocprof_avg_us(roof["rocprof_stats"], "cg_kernel")
    roof["rocprof_avg_launch_us"] = rp_us
    roof["spmv_frac_rocprof"] = (round(B * work / (rp_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)
                                 if rp_us else None)
    roof.update(cg_roofline_extras(B * work, B * cg_iter_work, avg_s, traffic))
    return {"B": B, "value": round(B * steps / elapsed, 3), "unit": "calls/s",
            "ms_per_step": round(1e3 * elapsed / steps, 4),
            "events_pass_ms_per_step": round(1e3 * elapsed_ev / steps, 4),
            "note": "one fwd+bwd of the batched entry point = B graphs, timed with no kernel "
                    "events; every CG launch timed by events carried in its dispatch packet in "
                    "a second pass (events_pass_ms_per_step)",
            "roofline": roof, "cg_iters_fwd_bwd": [it_f, it_b],
            "gram_mfma_pmc": gram_mfma_pmc(f"{c['name']}_b{B}")}


def c_abi_measure(X, Y, tau, eps, k, gbar, steps, warmup):
    """The same fwd+bwd through the C ABI of include/gll.h (gll_forward + gll_backward on the
    current stream, caller-owned workspace) without torch's autograd engine in the loop: what a
    native caller of the boundary gets, and the GPU-side rate of the step."""
    import ctypes as ct

    n, d = X.shape
    base, C = Y.shape
    prob = GLL.make_problem(n, d, base, C, k, tau, eps)
    lib = _lib.lib()
    ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device=X.device)
    U = torch.empty(n - base, C, dtype=torch.float64, device=X.device)
    gx = torch.empty(n, d, dtype=torch.float32, device=X.device)
    X32 = X.detach().contiguous()
    Yc = Y.contiguous()
    s = torch.cuda.current_stream(X.device).cuda_stream
    pp = ct.byref(prob)
    xp, yp, wp, up, gp, gxp = (X32.data_ptr(), Yc.data_ptr(), ws.data_ptr(), U.data_ptr(),
                               gbar.data_ptr(), gx.data_ptr())

    def step():
        lib.gll_forward(pp, xp, yp, _lib.GLL_DT_F32, wp, up, s)
        lib.gll_backward(pp, xp, None, 0, wp, gp, _lib.GLL_DT_F64, gxp, s)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"value": round(steps / el, 3), "unit": "calls/s", "ms_per_step": round(1e3 * el / steps, 4),
            "note": "same kernels and inputs through gll_forward + gll_backward (include/gll.h), "
                    "no torch autograd engine on the host path"}


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def _port_calibration():
    """Port-vs-reference time ratio measured in the build container, where the reference
    itself can run (tools/calibrate_port.py -> profiles/*_port_calibration.json)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_port_calibration.json")))
    if not paths:
        return None
    with open(paths[-1]) as f:
        doc = json.load(f)
    doc["file"] = os.path.relpath(paths[-1], ROOT)
    return doc


def cpu_baseline(cfg, eps, tau, seconds, config_name):
    """Time the reference's CPU step sequence (oracle/gll_port.py, 'port') on this host.

    Threads: torch's intra-op pool as the box sets it (OMP_NUM_THREADS = 16 = this job's CPU
    share on the GPU box, whatever nproc says); the port is mostly single-threaded anyway
    (SuperLU, scipy, the Python loop), like the reference."""
    from oracle import gll_port

    X, lab = synth(cfg["base"], cfg["batch"], cfg["d"], r=cfg["r"], seed=0)
    Y = torch.from_numpy(one_hot(lab[: cfg["base"]]))
    g = torch.from_numpy(seeded_gbar(cfg["batch"], 10))
    Xt = torch.from_numpy(X)
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        U, saved = gll_port.forward(Xt, Y, tau, eps, cfg["k"])
        gll_port.backward(saved, g)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    out = {"value": round(1.0 / med, 3), "unit": "calls/s", "cores": torch.get_num_threads(),
           "kind": "port",
           "sample": f"{len(times)} fwd+bwd calls of oracle/gll_port.py (reference step "
                     f"sequence: exact kNN + scipy CSR + SuperLU + torch sparse mm) on "
                     f"{cfg['base']}+{cfg['batch']}x{cfg['d']} k={cfg['k']}, median",
           "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
           "threads_note": ("torch intra-op threads = OMP_NUM_THREADS "
                            f"({os.environ.get('OMP_NUM_THREADS', 'unset')}), the job's CPU share "
                            "on the GPU box; nproc counts the whole host")}
    cal = _port_calibration()
    if cal is not None and config_name in cal.get("configs", {}):
        cc = cal["configs"][config_name]
        out["port_vs_reference"] = {
            "ratio_ref_over_port": cc["ratio_ref_over_port"],
            "port_ms": cc["port_ms"], "reference_ms": cc["reference_ms"],
            "where": cal.get("host", "build container"), "source": cal["file"],
            "reference_equiv_calls_s": round(out["value"] / cc["ratio_ref_over_port"], 3),
            "note": "reference = /root/reference/GLL.py with the exact graphlearning stand-in, "
                    "timed beside the port in the build container (the reference cannot travel "
                    "to the GPU box); reference_equiv = this box's port rate / ratio"}
    return out


def dry_run(a, world, rank):
    """CPU stand-in for the GPU leg (no measurement): the same launcher, warm-up/timed split,
    coalesced gather and max-over-ranks reduction, with a tiny deterministic CPU step whose
    'predictions' identify the rank, so the gathers can be checked for rank order."""
    if world > 1:
        dist.init_process_group("gloo")
    c = dict(CONFIGS["plumbing"])
    m = c["batch"]
    base_u = torch.arange(m * 10, dtype=torch.float64).reshape(m, 10) / (m * 10)
    gatherer = PredictionGatherer(every=GATHER_EVERY)

    def step(s):
        U = base_u + rank + 1000.0 * s
        gatherer.add(U)
        return U

    for s in range(a.warmup):
        step(s)
    gatherer.wait()
    gatherer.gathered = []
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(a.steps):
        step(a.warmup + s)
    gatherer.wait()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ok = True
    if world > 1:
        full = torch.cat([blk.transpose(0, 1) for blk in gatherer.gathered])   # (calls, world, m, C)
        for s in range(a.steps):
            for r in range(world):
                ok &= bool(torch.equal(full[s, r], base_u + r + 1000.0 * (a.warmup + s)))
        ok &= full.shape[0] == a.steps
    ident = rank_identity(None, torch.device("cpu"))   # outside the timed region
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "dry_run": True, "unit": "calls/s",
                          "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(1e3 * elapsed / max(a.steps, 1), 4),
                          "gather_check": "ok" if ok else "FAILED",
                          "ranks": ident, "distinct_gpus": distinct_devices(ident),
                          "config": {"workload": "dry-run stand-in", "parallelism": f"dp{world}"}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if ok else 1


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch(a)          # N ranks, one per GPU; nothing here has touched the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if a.dry_run:
        return dry_run(a, world, rank)
    if a.share_gpu:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if a.share_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    coll = torch.device("cpu") if a.share_gpu else dev   # gloo collectives on host tensors

    c = dict(CONFIGS[a.config])
    c["n"] = c["base"] + c["batch"]
    c["name"] = a.config
    eps, tau, k = EPS[a.config], TAU[a.config], c["k"]
    X_np, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=shard_rank_seed(0, rank))
    X = torch.from_numpy(X_np).to(dev).requires_grad_(True)
    Y = torch.from_numpy(one_hot(lab[: c["base"]])).to(dev)
    gbar = torch.from_numpy(seeded_gbar(c["batch"], 10, 1234 + rank)).to(dev)
    lap = GLL.LaplaceLearningSparseHard.apply

    gatherer = PredictionGatherer(every=GATHER_EVERY, keep=1)

    def step():
        U = lap(X, Y, tau, eps, k)
        gatherer.add(U)          # one async RCCL all_gather per GATHER_EVERY calls
        (gx,) = torch.autograd.grad(U, X, gbar)
        return U, gx

    for _ in range(a.warmup):
        step()
    gatherer.wait()
    torch.cuda.synchronize()

    # which kernel dominates: one untimed instrumented pass over all kernels
    names = [_lib.kernel_name(q) for q in range(_lib.K_COUNT)]
    per_kernel = {}
    dominant = None
    if not a.no_profile:
        for q in range(_lib.K_COUNT):
            _lib.prof_enable(q, 1)
        # as many bracketed steps as the timed region will sample, so that every event pair it
        # uses comes from the pool these leave behind: a hipEventCreate inside the timed region
        # cost ~12 us each (every 7th step brackets 5 kernels: 17 us per step on average,
        # profiles/r04v_bench_ns.json against r04a)
        n_inst = max(10, a.steps // PROF_PERIOD + 2)
        for _ in range(n_inst):
            step()
        gatherer.wait()
        torch.cuda.synchronize()
        for q in range(_lib.K_COUNT):
            ms, cnt = _lib.prof_read(q)
            _lib.prof_enable(q, 0)
            if cnt:
                per_kernel[names[q]] = {"us_per_launch": round(1e3 * ms / cnt, 3),
                                        "launches_per_step": cnt / n_inst}
        dominant = max(per_kernel, key=lambda kn: per_kernel[kn]["us_per_launch"]
                       * per_kernel[kn]["launches_per_step"])

    # timed region (the backward on the thread --autograd-thread names: on a host whose torch
    # engine hand-off to its device thread costs more than the step's GPU work -- ~40 us per
    # call on some boxes, profiles/r04a_host_breakdown.txt -- the calling thread keeps the
    # step GPU-bound; the other mode is timed after the run and reported beside it)
    probe = None
    if a.autograd_thread == "auto":
        # untimed: short runs of each mode, alternated twice and the faster run of each kept --
        # the first run in device mode pays the engine's thread start-up, and a single pass
        # picked caller mode (66.9 vs 69.8 us) on a box where device mode then timed 62.8 us
        # against caller's 66.5 (profiles/r06k_bench_ns.json); the faster mode is timed below
        # and the other reported beside it
        probe = {}
        for mode in ("caller", "device", "caller", "device"):
            with torch.autograd.set_multithreading_enabled(mode == "device"):
                for _ in range(min(a.warmup, 5)):
                    step()
                gatherer.wait()
                torch.cuda.synchronize()
                t0_ = time.perf_counter()
                for _ in range(min(a.steps, 100)):
                    step()
                gatherer.wait()
                torch.cuda.synchronize()
                ms_ = round(1e3 * (time.perf_counter() - t0_) / min(a.steps, 100), 4)
                probe[mode] = min(probe.get(mode, ms_), ms_)
        a.autograd_thread = min(probe, key=probe.get)
    mt = torch.autograd.set_multithreading_enabled(a.autograd_thread == "device")
    mt.__enter__()
    for _ in range(min(a.warmup, 5)):   # untimed: the first steps in this mode
        step()
    gatherer.wait()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        U, gx = step()
    gatherer.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the kernels' live launch times: a second pass of a.steps steps right after, the same step
    # and engine mode, with HIP events in the dispatch packets of every PROF_PERIOD-th launch of
    # every kernel (each runs once per step here, so the same steps; a kernel whose predecessor on
    # the stream carries no event reads up to 2 us long, profiles/r04g_path_probe.txt "cgonly").
    # The headline pass above carries no events: they cost the NS step 5.5% (15.05K against
    # 15.86K calls/s, alternating runs on one box, profiles/r06r_events_ab.txt).
    events_pass = None
    if dominant is not None:
        for q in range(_lib.K_COUNT):
            _lib.prof_read(q)
            _lib.prof_enable(q, PROF_PERIOD)
        torch.cuda.synchronize()
        t0_ = time.perf_counter()
        for _ in range(a.steps):
            step()
        gatherer.wait()
        torch.cuda.synchronize()
        events_pass = {"steps": a.steps, "ms_per_step": round(1e3 * (time.perf_counter() - t0_) / a.steps, 4),
                       "period": PROF_PERIOD,
                       "note": "the pass the kernel events (roofline, kernels) come from; the "
                               "headline pass carries none"}
    mt.__exit__(None, None, None)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # which GPU each rank ran on, as the process group sees it (one tiny all_gather, outside the
    # timed region): a scaling line carries its own proof of N distinct devices and N ranks
    ident = rank_identity(dev, coll)
    distinct = distinct_devices(ident)
    if world > 1 and not distinct and not a.share_gpu and rank == 0:
        print(f"bench.py: ranks did not report {world} distinct GPUs: {ident}", file=sys.stderr)

    gather_check = None
    if world > 1:
        # every rank's inputs are fixed, so each slot of the last gathered group must hold
        # that rank's U: compare per-rank checksums (one tiny all_gather, outside the timing)
        own = U.detach().double().sum().reshape(1).to(coll)
        sums = torch.empty(world, dtype=torch.float64, device=coll)
        dist.all_gather_into_tensor(sums, own)
        sums = sums.to(dev)
        blk = gatherer.gathered[-1].double().sum(dim=(2, 3))            # (world, calls)
        gather_check = "ok" if torch.allclose(blk, sums[:, None].expand_as(blk),
                                              rtol=1e-12, atol=0.0) else "FAILED"

    roofline = None
    call_roof_s = None
    if dominant is not None:
        ms, cnt = _lib.prof_read(names.index(dominant))
        for q in range(_lib.K_COUNT):
            _lib.prof_enable(q, 0)
            _lib.prof_read(q)
        g = GLL.device_graph(X.detach(), k, eps)
        rp = g["row_ptr"].cpu().numpy()
        col = g["col"].cpu().numpy()
        rows = np.repeat(np.arange(c["n"]), np.diff(rp))
        nnz_uu = int(np.sum((rows >= c["base"]) & (col >= c["base"])))
        GLL.check_status()
        iters = _cg_iters(X, Y, tau, eps, k, gbar)
        gstats = (int(rp[-1]), nnz_uu)
        units = kernel_units(c, gstats, iters[0], iters[1], isinstance(eps, str))
        cg_iter_work = cg_iteration_bytes(c, gstats, iters[0], iters[1])
        bound, work = units[dominant]
        avg_s = ms / cnt / 1e3
        if bound == "mfma":
            achieved, peak, unit = work / avg_s / 1e12, GRAM_ROOF_TFS, "TFLOP/s"
        else:
            achieved, peak, unit = work / avg_s / 1e9, HBM_PEAK_GBS, "GB/s"
        traffic = pmc_traffic(a.config, dominant)
        roofline = {"kernel": dominant, "bound": bound, "achieved": round(achieved, 3),
                    "peak": peak, "unit": unit, "frac": round(achieved / peak, 5),
                    "traffic": traffic, "work_per_launch": work,
                    "avg_launch_us": round(avg_s * 1e6, 3), "launches": cnt,
                    "cg_iters_fwd_bwd": list(iters),
                    "gram_mfma_pmc": gram_mfma_pmc(a.config),
                    "rocprof_stats": rocprof_stats(a.config)}
        rp_us = rocprof_avg_us(roofline["rocprof_stats"], dominant)
        roofline["rocprof_avg_launch_us"] = rp_us
        roofline["frac_rocprof"] = (round((work / (rp_us * 1e-6) / (1e12 if bound == "mfma" else 1e9))
                                          / peak, 5) if rp_us else None)
        if dominant == "cg_kernel":
            roofline["definition"] = ("SURVEY §8d SpMV roofline: B_spmv x iterations / CG launch "
                                      "time / 8 TB/s, B_spmv = 8 nnz_off(Luu) + 8 m + 8 m C")
            roofline["spmv_frac"] = roofline["frac"]
            roofline.update(cg_roofline_extras(work, cg_iter_work, avg_s, traffic))
        # SURVEY §8d's SpMV roofline of the forward CG launch (reported whatever kernel dominates;
        # the backward's CG may run inside the fused backward launch)
        if "cg_kernel" in per_kernel:
            t_cg = per_kernel["cg_kernel"]["us_per_launch"] * 1e-6
            w_cg = units["cg_kernel"][1]
            roofline["sec8d_cg_spmv"] = {
                "kernel": "cg_kernel", "work_per_launch": w_cg, "us_per_launch": round(t_cg * 1e6, 3),
                "achieved_GBs": round(w_cg / t_cg / 1e9, 3),
                "frac": round(w_cg / t_cg / 1e9 / HBM_PEAK_GBS, 5),
                "note": "B_spmv x iterations / launch time / 8 TB/s; a single NS graph is "
                        "latency-bound (SURVEY §7: 30% would need 29 ns per SpMV) -- the batched "
                        "line below carries the meaningful SpMV figure"}
        # whole-call roofline: kNN at its MFMA roof + every other byte at HBM,
        # a CG priced per whole iteration (B_spmv + 28 mC)
        f_knn = units["gram_d2_kernel"][1]
        call_units = dict(units)
        call_units["cg_kernel"] = ("hbm", cg_iter_work)
        b_rest = sum(w_ * per_kernel[kn]["launches_per_step"] for kn, (b_, w_) in call_units.items()
                     if b_ == "hbm" and kn in per_kernel)
        call_roof_s = {  # SURVEY §8d prices the kNN at the fp32 MFMA peak; the split-bf16 roof
                         # is what the Gram here actually runs on (both reported, labelled)
            "fp32_mfma": f_knn / (MFMA_F32_PEAK_TFS * 1e12) + b_rest / (HBM_PEAK_GBS * 1e9),
            "split_bf16": f_knn / (GRAM_ROOF_TFS * 1e12) + b_rest / (HBM_PEAK_GBS * 1e9)}
        for kn, v in per_kernel.items():
            b_, w_ = units[kn]
            v["algorithmic"] = (f"{w_ / 1e9:.4g} GFLOP" if b_ == "mfma" else f"{w_ / 1e6:.4g} MB")
            # each kernel against its own roof (SURVEY §8d units over its live launch time): the
            # Gram on the split-bf16 MFMA roof, everything else on 8 TB/s of HBM
            t_ = v["us_per_launch"] * 1e-6
            if t_ > 0:
                v["roofline_frac"] = round(w_ / t_ / 1e12 / GRAM_ROOF_TFS if b_ == "mfma"
                                           else w_ / t_ / 1e9 / HBM_PEAK_GBS, 5)
                pt = pmc_traffic(a.config, kn)
                if pt:
                    v["pmc_traffic_over_algorithmic"] = round(pt / w_, 3) if b_ == "hbm" else None

    c_abi = None
    if not a.no_profile:
        c_abi = c_abi_measure(X, Y, tau, eps, k, gbar, a.steps, a.warmup)

    # the same step with the autograd engine's other threading mode (labelled, not `value`)
    other = None
    if world == 1 and not a.no_profile:
        with torch.autograd.set_multithreading_enabled(a.autograd_thread != "device"):
            for _ in range(a.warmup):
                step()
            torch.cuda.synchronize()
            t0_ = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            el_ = time.perf_counter() - t0_
        other = {"autograd_thread": "device" if a.autograd_thread != "device" else "caller",
                 "value": round(a.steps / el_, 3), "unit": "calls/s",
                 "ms_per_step": round(1e3 * el_ / a.steps, 4),
                 "note": "the same apply + autograd.grad step with torch's other engine threading"}

    # the adversarial scripts' inline-copy call (train_and_adversarial.py:721,745;
    # adversarial.py:534): lap(features, one_hot(labels)[:k]) -- int64 labels, tau = 0, eps =
    # 'auto' -- on the same graph, through apply + autograd.grad (labelled extra, not `value`)
    auto_extra = None
    if a.config == "ns" and not a.no_profile and world == 1:
        Yi = Y.to(torch.int64)
        per_k = {}

        def step_auto_k():
            U_ = lap(X, Yi, 0, "auto", k)
            return torch.autograd.grad(U_, X, gbar)

        for fn_ in (step_auto_k,):
            for _ in range(a.warmup):
                fn_()
            torch.cuda.synchronize()
            for q in range(_lib.K_COUNT):
                _lib.prof_enable(q, 1)
            for _ in range(10):
                fn_()
            torch.cuda.synchronize()
            for q in range(_lib.K_COUNT):
                ms_, cnt_ = _lib.prof_read(q)
                _lib.prof_enable(q, 0)
                if cnt_:
                    per_k[names[q]] = {"us_per_launch": round(1e3 * ms_ / cnt_, 3),
                                       "launches_per_step": cnt_ / 10}
            torch.cuda.synchronize()
            t0_ = time.perf_counter()
            for _ in range(a.steps):
                fn_()
            torch.cuda.synchronize()
            el_ = time.perf_counter() - t0_
        GLL.check_status()
        auto_extra = {"call": f"lap(X, one_hot int64, tau=0, epsilon='auto', k={k})",
                      "reference": "train_and_adversarial.py:721,745; adversarial.py:534",
                      "value": round(a.steps / el_, 3), "unit": "calls/s",
                      "ms_per_step": round(1e3 * el_ / a.steps, 4), "kernels": per_k,
                      "note": "same NS graph inputs as the headline, the inline-copy callers' "
                              "epsilon / tau / label dtype (k kept at the workload's 10)"}

    batched = None
    if a.batch > 0 and roofline is not None:
        batched = batched_measure(c, eps, tau, k, a.batch, gstats, dev, rank)

    cpu = None
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        cpu = cpu_baseline(c, eps, tau, a.cpu_seconds, a.config)

    if rank == 0:
        calls = world * a.steps
        # every GLL_* variable of this process: the product library reads only GLL_DEBUG (it
        # prints launch errors); GLL_LIB_PATH loads another build (A/B), so no value is reported
        gll_env = {kk: vv for kk, vv in sorted(os.environ.items()) if kk.startswith("GLL_")}
        foreign = sorted(kk for kk in gll_env if kk not in ("GLL_DEBUG",))
        out = {
            "metric": METRIC,
            "value": None if foreign else round(calls / elapsed, 3),
            "unit": "calls/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * elapsed / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (latent-mixture unit-norm features, SURVEY.md §8d; seed = rank)",
            "config": {"workload": a.config, "base": c["base"], "batch": c["batch"], "d": c["d"],
                       "k": k, "eps": eps, "tau": tau, "classes": 10,
                       "parallelism": f"dp{world}", "upstream_grad": "fixed seeded dL/dU",
                       # the autograd engine's threading mode the value was timed in (part of the
                       # workload's identity: compare lines across rounds only at equal modes)
                       "autograd_thread": a.autograd_thread,
                       "collective": (("gloo all_gather(U) staged through the host, one per "
                                       f"{GATHER_EVERY} calls" if a.share_gpu else
                                       f"async all_gather(U) over RCCL, one per {GATHER_EVERY} calls")
                                      if world > 1 else "none")},
            "roofline": roofline,
            "events_pass": events_pass,
            "cpu_baseline": cpu,
            "gather_check": gather_check,
            "ranks": ident,
            "distinct_gpus": distinct,
            "kernels": per_kernel,
            "c_abi": c_abi,
            "autograd_thread": (a.autograd_thread + (" (torch.autograd.set_multithreading_enabled("
                                f"{a.autograd_thread == 'device'}))")),
            "autograd_other_thread": other,
            "autograd_probe_ms_per_step": probe,
            "batched": batched,
            "auto_eps_extra": auto_extra,
            "gll_env": gll_env,
            "build_id": _lib.build_id(),
            "profiles_of_this_build": build_profile_tags(),
        }
        if foreign:
            out["invalid"] = (f"GLL_* variables that change what runs are set ({', '.join(foreign)}): "
                              "not a measurement of the product library")
        if roofline is not None:
            step_s = elapsed / a.steps
            out["call_roofline"] = {
                "definition": "t_roof = F_kNN / MFMA peak + B_rest / 8 TB/s (SURVEY.md §8d), "
                              "frac = t_roof / measured step time",
                "sec8d_fp32_mfma": {"kNN_peak_TFs": MFMA_F32_PEAK_TFS,
                                    "t_roof_us": round(call_roof_s["fp32_mfma"] * 1e6, 3),
                                    "frac": round(call_roof_s["fp32_mfma"] / step_s, 5)},
                "split_bf16": {"kNN_peak_TFs": round(GRAM_ROOF_TFS, 1),
                               "t_roof_us": round(call_roof_s["split_bf16"] * 1e6, 3),
                               "frac": round(call_roof_s["split_bf16"] / step_s, 5)}}
        if cpu:
            out["speedup_vs_cpu"] = round(out["value"] / cpu["value"], 1)
        if a.share_gpu:
            out["share_gpu"] = (f"DIAGNOSTIC: all {world} ranks ran on cuda:0 over gloo -- the "
                                "real apply / gather / timed-region code of the multi-rank leg on "
                                "a one-GPU box; value is not a scaling measurement")
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _cg_iters(X, Y, tau, eps, k, gbar):
    """CG iterations (max over columns) of one fwd and one bwd solve on the bench input
    (X: n x d, or B x n x d through the batched entry points: graph 0's solves)."""
    import ctypes as ct

    B = X.shape[0] if X.dim() == 3 else 1
    n, d = X.shape[-2:]
    base, C = Y.shape[-2:]
    prob = GLL.make_problem(n, d, base, C, k, tau, eps)
    lib = _lib.lib()
    nb = lib.gll_workspace_bytes(ct.byref(prob))
    ws = torch.empty(nb * B, dtype=torch.uint8, device=X.device)
    U = torch.empty(B, n - base, C, dtype=torch.float64, device=X.device)
    X32 = X.detach().contiguous()
    Yc = Y.contiguous()
    s = torch.cuda.current_stream(X.device).cuda_stream
    _lib.check(lib.gll_forward_batched(ct.byref(prob), B, X32.data_ptr(), Yc.data_ptr(),
                                       _lib.GLL_DT_F32, ws.data_ptr(), U.data_ptr(), s),
               "gll_forward")
    gx = torch.empty(B, n, d, dtype=torch.float32, device=X.device)
    _lib.check(lib.gll_backward_batched(ct.byref(prob), B, X32.data_ptr(), ws.data_ptr(),
                                        gbar.contiguous().data_ptr(), _lib.GLL_DT_F64,
                                        gx.data_ptr(), s), "gll_backward")
    st = ws[: 4 * _lib.ST_NWORDS].view(torch.int32).cpu().tolist()
    return st[_lib.ST_FWD_ITERS], st[_lib.ST_BWD_ITERS]


if __name__ == "__main__":
    sys.exit(main())
