"""Time oracle/gll_port.py beside the REFERENCE GLL.py in the build container (CPU only).

    python tools/calibrate_port.py [--out profiles/r02_port_calibration.json]

bench.py's cpu_baseline times the port on the GPU box because /root/reference does not
travel there; this records, per config, how the port's time relates to the reference's on
the same host and inputs, so the box's port number can be read as a reference number.
The reference is /root/reference/GLL.py imported as-is with the exact graphlearning
stand-in (tests/golden/make_golden.py: load_reference); k is overridden through the module
global knn_sym_dist, as there.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402
from oracle import gll_port  # noqa: E402

EPS = {"plumbing": 1.0, "ns": 1.0, "fullysup": 1.0, "stress": "auto"}
REPS = {"plumbing": 20, "ns": 10, "fullysup": 6, "stress": 2}


def _cpu_model():
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    return "?"


def time_calls(fn, reps):
    fn()                                  # warm-up
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_port_calibration.json"))
    ap.add_argument("--configs", default="plumbing,ns,fullysup,stress")
    a = ap.parse_args()
    from make_golden import load_reference
    ref = load_reference()
    orig = ref.knn_sym_dist
    out = {"host": f"build container: {_cpu_model()}, nproc {os.cpu_count()}",
           "torch_threads": torch.get_num_threads(), "configs": {}}
    for name in a.configs.split(","):
        c = CONFIGS[name]
        X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
        Y = torch.from_numpy(one_hot(lab[: c["base"]]))
        g = torch.from_numpy(seeded_gbar(c["batch"], 10))
        eps, tau, k = EPS[name], 0.07, c["k"]

        def port():
            U, saved = gll_port.forward(torch.from_numpy(X), Y, tau, eps, k)
            gll_port.backward(saved, g)

        def reference():
            ref.knn_sym_dist = lambda data, k=25, epsilon="auto": orig(data, k=c["k"], epsilon=epsilon)
            try:
                Xt = torch.from_numpy(X).requires_grad_(True)
                U = ref.LaplaceLearningSparseHard.apply(Xt, Y, tau, eps)
                U.backward(g)
            finally:
                ref.knn_sym_dist = orig

        tp = time_calls(port, REPS[name])
        tr = time_calls(reference, REPS[name])
        out["configs"][name] = {"port_ms": round(tp, 2), "reference_ms": round(tr, 2),
                                "ratio_ref_over_port": round(tr / tp, 3), "reps": REPS[name],
                                "eps": eps, "tau": tau, "k": k}
        print(name, out["configs"][name], flush=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
