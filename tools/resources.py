"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` output: one line per kernel."""
import re
import subprocess
import sys

log = open(sys.argv[1]).read() if len(sys.argv) > 1 else sys.stdin.read()
cur = None
rows = []
for line in log.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass-analysis", line)
    if not m:
        continue
    kv = m.group(1)
    if kv.startswith("Function Name:"):
        cur = {"name": kv.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in kv:
        k, v = kv.split(":", 1)
        cur[k.strip()] = v.strip()
names = [r["name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    d = re.sub(r"\(.*", "", d).replace("gll::", "")
    print(f"{d:45s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>4} "
          f"scratch={r.get('ScratchSize [bytes/lane]','?'):>4} occ={r.get('Occupancy [waves/SIMD]','?')} "
          f"lds={r.get('LDS Size [bytes/block]','?')}")
