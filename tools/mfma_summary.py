"""MFMA utilisation per kernel from a rocprofv3 --pmc pass (diagnostic, run on the profile dirs).

usage: python tools/mfma_summary.py <pmc_dir> <out.json> [--label NAME]

The pass collects SQ_INSTS_VALU_MFMA_MOPS_BF16 (bf16 MFMA flops / 512), SQ_VALU_MFMA_BUSY_CYCLES
(cycles an MFMA unit is busy, summed over the SIMDs), SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE (summed
over the 8 XCDs) with --kernel-trace.  Per launch of each kernel:
  executed bf16 TFLOP/s = MOPS x 512 / duration           (duration from the same pass's trace)
  flops % of peak       = executed TFLOP/s / 2500          (dense bf16, MI355X_MICROARCH.md)
  MFMA busy %           = BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
The split-bf16 Gram executes 3 bf16 products per fp32 product over its tile schedule, so its
algorithmic rate (2 n^2 d / duration) is reported by bench.py, not here.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
BF16_PEAK_TFS = 2500.0


def short(name):
    name = name.split("(")[0]
    if name.startswith("void "):
        name = name[5:]
    return name.split("<")[0].split("::")[-1]


def main():
    args = sys.argv[1:]
    label = None
    if "--label" in args:
        i = args.index("--label")
        label = args[i + 1]
        del args[i:i + 2]
    d, out = args
    vals = defaultdict(lambda: defaultdict(list))
    disp = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                disp.setdefault(k, []).append(
                    (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    kernels = {}
    for k, cs in vals.items():
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        dur = sum(disp.get(k, [0])) / max(1, len(disp.get(k, [])))
        e = {"launches": len(next(iter(cs.values()))), "duration_us": round(dur * 1e6, 3)}
        e.update({c: round(v, 1) for c, v in mean.items()})
        mops = mean.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0)
        if mops and dur:
            e["exec_bf16_tflops"] = round(mops * 512 / dur / 1e12, 2)
            e["exec_flops_frac_of_peak"] = round(mops * 512 / dur / 1e12 / BF16_PEAK_TFS, 4)
        busy, gui = mean.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), mean.get("GRBM_GUI_ACTIVE", 0.0)
        if busy and gui:
            e["mfma_busy_frac"] = round(busy / (SIMDS * gui / 8.0), 4)
            if dur:
                e["clock_ghz_from_gui"] = round(gui / 8.0 / dur / 1e9, 3)
        kernels[k] = e
    doc = {"label": label, "source": "rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 "
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace",
           "unit": "per launch (mean)", "kernels": kernels}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k, e in sorted(kernels.items()):
        if "exec_bf16_tflops" in e or "mfma_busy_frac" in e:
            print(f"{k:24s} {e['duration_us']:9.2f} us  exec {e.get('exec_bf16_tflops', 0):8.1f} TF/s"
                  f"  ({100 * e.get('exec_flops_frac_of_peak', 0):5.1f}% of bf16 peak)"
                  f"  MFMA busy {100 * e.get('mfma_busy_frac', 0):5.1f}%")


if __name__ == "__main__":
    main()
