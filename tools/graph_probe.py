"""kNN graph only (Gram + select + row build through gll_graph), repeated: a profiling target
for the Gram's MFMA counters at a config's shape without the solves (diagnostic, GPU box).

    PROBE_CFG=stress python tools/graph_probe.py
"""
import ctypes as ct
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd import GLL, _lib  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, synth  # noqa: E402

cfg = os.environ.get("PROBE_CFG", "stress")
reps = int(os.environ.get("PROBE_REPS", "10"))
c = CONFIGS[cfg]
n = c["base"] + c["batch"]
X, _ = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=0)
dev = torch.device("cuda", 0)
Xd = torch.from_numpy(X).to(dev)
prob = GLL.make_problem(n, c["d"], 0, 1, c["k"], 0.0, "auto")
lib = _lib.lib()
ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(reps):
    _lib.check(lib.gll_graph(ct.byref(prob), Xd.data_ptr(), ws.data_ptr(), s), "gll_graph")
torch.cuda.synchronize()
print(f"{cfg}: {reps} graphs built (n={n}, d={c['d']}, k={c['k']})")
