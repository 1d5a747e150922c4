"""Time the reference's per-step base draw against the device-resident provider (§8f-4).

    python tools/base_loader_probe.py [--n 250] [--workers 0,2,4] [--reps 20]

(a) the reference pattern: `next(iter(DataLoader(base_set, batch_size=N, shuffle=True,
    num_workers=W, pin_memory=True)))` then `.cuda(non_blocking=True)` (FullySup.py:135-143,
    loader built at FullySup.py:262-266), on CIFAR-shaped synthetic images (3 x 32 x 32 fp32,
    the ToTensor output select_base_data stacks, utils.py:796-806);
(b) graphlearninglayer_amd.base_data.DeviceBaseLoader.sample() on the GPU.
Prints one JSON line per variant (median ms per draw, device-synchronised).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd.base_data import DeviceBaseLoader  # noqa: E402


class CustomDataset(torch.utils.data.Dataset):   # the shape of utils.py:170-187, transform=None
    def __init__(self, data, labels):
        self.data, self.labels = data, labels

    def __len__(self):
        return len(self.data)

    def __getitem__(self, i):
        return self.data[i], self.labels[i]


def med_ms(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=250)
    ap.add_argument("--workers", default="0,2,4")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    data = torch.rand(a.n, 3, 32, 32, generator=g)
    labels = torch.arange(a.n) % 10
    ds = CustomDataset(data, labels)
    for w in [int(x) for x in a.workers.split(",")]:
        dl = torch.utils.data.DataLoader(ds, batch_size=len(ds), shuffle=True, num_workers=w,
                                         pin_memory=True)

        def ref_draw():
            im, lb = next(iter(dl))
            return im.cuda(non_blocking=True), lb.cuda(non_blocking=True)

        print(json.dumps({"variant": f"DataLoader next(iter()) + .cuda(), num_workers={w}",
                          "n": a.n, "ms_per_draw": round(med_ms(ref_draw, a.reps), 4)}), flush=True)
    p = DeviceBaseLoader(data, labels, device="cuda", seed=0)
    print(json.dumps({"variant": "DeviceBaseLoader.sample() (HBM-resident, on-device randperm)",
                      "n": a.n, "ms_per_draw": round(med_ms(p.sample, max(a.reps, 200)), 4)}),
          flush=True)


if __name__ == "__main__":
    main()
