"""How often the select kernel's exact candidate merge runs (GLL_ST_KNN_MERGE) per config
(diagnostic, GPU box): rows whose short per-lane lists may have dropped a column."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, synth  # noqa: E402

for name in sys.argv[1:] or ["ns", "fullysup", "stress"]:
    c = CONFIGS[name]
    X, _ = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
    g = GLL.device_graph(torch.from_numpy(X).cuda(), c["k"], "auto")
    st = g["status"].cpu()
    print(f"{name}: n={X.shape[0]} k={c['k']} merge={int(st[_lib.ST_KNN_MERGE])} "
          f"rescan={int(st[_lib.ST_KNN_RESCAN])}", flush=True)
