"""Per-workgroup dispatch of the Gram kernel (diagnostic, GPU box, trace build).

For GLL_GRAM_KS in the environment, runs forwards at NS and prints how many workgroups were
resident over time, per-XCD / per-CU placement and per-workgroup durations.
"""
import ctypes as ct
import os
import sys
from collections import Counter

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from graphlearninglayer_amd import GLL  # noqa: E402
from graphlearninglayer_amd.synth import CONFIGS, one_hot, synth  # noqa: E402

lib = ct.CDLL(os.path.join(ROOT, "graphlearninglayer_amd", "_obj", "libgll_trace.so"))
lib.gll_workspace_bytes.restype = ct.c_size_t
c = CONFIGS[os.environ.get("TRACE_CFG", "ns")]
n, base, d, k = c["base"] + c["batch"], c["base"], c["d"], c["k"]
dev = torch.device("cuda", 0)
X_np, lab = synth(base, n - base, d, r=c["r"], seed=0)
X = torch.from_numpy(X_np).to(dev)
Y = torch.from_numpy(one_hot(lab[:base])).to(dev)
prob = GLL.make_problem(n, d, base, 10, k, 0.07, 1.0)
ws = torch.empty(lib.gll_workspace_bytes(ct.byref(prob)), dtype=torch.uint8, device=dev)
U = torch.empty(n - base, 10, dtype=torch.float64, device=dev)
s = ct.c_void_p(torch.cuda.current_stream().cuda_stream)
T = (n + 63) // 64
nwg = T * (T + 1) // 2 * int(os.environ.get("GLL_GRAM_KS", "1"))
for _ in range(10):
    lib.gll_forward(ct.byref(prob), ct.c_void_p(X.data_ptr()), ct.c_void_p(Y.data_ptr()), 0,
                    ct.c_void_p(ws.data_ptr()), ct.c_void_p(U.data_ptr()), s)
torch.cuda.synchronize()
KERNEL = int(os.environ.get("PROBE_KERNEL", "0"))   # 0 gram, 1 select
if KERNEL == 1:
    nwg = (n + 3) // 4
buf = (ct.c_ulonglong * (2 * 3 * 4096))()
lib.gll_trace_read_wg(0, buf)
a = np.array(buf[:], dtype=np.uint64).astype(np.int64).reshape(2, 3, 4096)[KERNEL][:, :nwg]
ent, ext, cu = a[0], a[1], a[2]
t0 = ent.min()
ent = (ent - t0) / 100.0
ext = (ext - t0) / 100.0
print(f"kernel {KERNEL} workgroups {nwg}: entry spread {ent.max():.2f} us, last exit {ext.max():.2f} us, "
      f"duration mean {np.mean(ext - ent):.2f} min {np.min(ext - ent):.2f} max {np.max(ext - ent):.2f}")
dur = ext - ent
print("duration percentiles (us) 10/50/90/99/max:",
      " ".join(f"{np.percentile(dur, q):.2f}" for q in (10, 50, 90, 99, 100)))
print("slowest 8 workgroups:", " ".join(f"{int(b)}:{dur[b]:.1f}" for b in np.argsort(dur)[-8:]))
for t in np.arange(0, ext.max() + 1, 1.0):
    print(f"  t={t:5.1f} resident {int(np.sum((ent <= t) & (ext > t)))}")
xcc = cu >> 6
print("per XCD:", dict(sorted(Counter(xcc.tolist()).items())))
print("distinct CU ids:", len(set(cu.tolist())), " max WGs on one CU id:",
      max(Counter(cu.tolist()).values()))
order = np.argsort(ent)
print("first 16 by entry: " + " ".join(f"{int(b)}@{ent[b]:.1f}/x{int(xcc[b])}" for b in order[:16]))
print("last 16 by entry: " + " ".join(f"{int(b)}@{ent[b]:.1f}/x{int(xcc[b])}" for b in order[-16:]))
