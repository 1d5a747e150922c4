cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && R=$PWD
P="timeout -s KILL 120 rocprofv3"
GS="python3 $R/tools/graph_probe.py"
export PROBE_CFG=stress
$P --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pk_fetch -o run -- $GS > gpurun_out/pk_fetch.log 2>&1 && \
$P --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pk_hit -o run -- $GS > gpurun_out/pk_hit.log 2>&1 && \
$P --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pk_mfma -o run -- $GS > gpurun_out/pk_mfma.log 2>&1
echo rc=$?
python3 tools/mfma_summary.py gpurun_out/pk_mfma gpurun_out/pk_mfma.json --label stress_pk
python3 - <<'PY'
import csv,glob,collections
for d,cs in (("gpurun_out/pk_fetch",["FETCH_SIZE"]),("gpurun_out/pk_hit",["TCC_HIT_sum","TCC_MISS_sum"])):
    acc=collections.defaultdict(list)
    for p in glob.glob(d+"/**/*counter_collection.csv",recursive=True):
        for r in csv.DictReader(open(p)):
            acc[(r["Kernel_Name"].split("(")[0][-40:],r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k,v in sorted(acc.items()): print(k, round(sum(v)/len(v),1), len(v))
PY
