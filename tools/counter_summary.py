"""Per-kernel averages of every counter in a rocprofv3 --pmc run directory (counter_collection.csv):
one line per kernel, counter values summed over the dimensions of one dispatch, then averaged over
its dispatches."""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))   # (kernel, dispatch) -> counter
for row in csv.DictReader(open(f)):
    name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void ", "").replace("gll::", "")
    per[(name, row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for (name, _), cs in per.items():
    for k, v in cs.items():
        agg[name][k].append(v)
for name, cs in sorted(agg.items()):
    vals = {k: sum(v) / len(v) for k, v in cs.items()}
    n = len(next(iter(cs.values())))
    line = " ".join(f"{k}={v:.4g}" for k, v in sorted(vals.items()))
    extra = ""
    if vals.get("SQ_LDS_IDX_ACTIVE"):
        extra = f" | conflict/idx_active={vals.get('SQ_LDS_BANK_CONFLICT', 0) / vals['SQ_LDS_IDX_ACTIVE']:.3f}"
    print(f"{name[:60]:60s} n={n} {line}{extra}")
