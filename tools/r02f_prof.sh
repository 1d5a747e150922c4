# Round-2 final profile session (GPU box): rocprof kernel stats + FETCH/WRITE PMC for NS B=64,
# FullySup B=64 and stress, Gram MFMA counters at stress and NS B=64, FullySup single-graph stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && R=$PWD
P="timeout -s KILL 150 rocprofv3"
MF="--pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv"
ST="python3 $R/bench.py --config stress --steps 10 --warmup 3 --cpu-seconds 0 --no-profile --batch 0"
FS="python3 $R/bench.py --config fullysup --steps 100 --warmup 10 --cpu-seconds 0 --no-profile --batch 0"
B64="python3 $R/tools/batch_probe.py"
export PROBE_B=64 GLL_GRID_COOP=0
$P --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b64 -o run -- $B64 > gpurun_out/prof_b64.log 2>&1 && \
$P --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_b64 -o run -- $B64 > gpurun_out/pmc_fetch_b64.log 2>&1 && \
$P --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_b64 -o run -- $B64 > gpurun_out/pmc_write_b64.log 2>&1 && \
PROBE_CFG=fullysup $P --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fs64 -o run -- $B64 > gpurun_out/prof_fs64.log 2>&1 && \
PROBE_CFG=fullysup $P --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_fs64 -o run -- $B64 > gpurun_out/pmc_fetch_fs64.log 2>&1 && \
PROBE_CFG=fullysup $P --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_fs64 -o run -- $B64 > gpurun_out/pmc_write_fs64.log 2>&1 && \
$P --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stress -o run -- $ST > gpurun_out/prof_stress.log 2>&1 && \
$P --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_stress -o run -- $ST > gpurun_out/pmc_fetch_stress.log 2>&1 && \
$P --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_stress -o run -- $ST > gpurun_out/pmc_write_stress.log 2>&1 && \
PROBE_CFG=stress $P $MF -d $R/gpurun_out/mfma_stress -o run -- python3 $R/tools/graph_probe.py > gpurun_out/mfma_stress.log 2>&1 && \
$P $MF -d $R/gpurun_out/mfma_b64 -o run -- $B64 > gpurun_out/mfma_b64.log 2>&1 && \
$P --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fullysup -o run -- $FS > gpurun_out/prof_fullysup.log 2>&1
rc=$?
echo "profile session rc=$rc"
for x in b64 stress; do [[ -d gpurun_out/mfma_$x ]] && python3 tools/mfma_summary.py gpurun_out/mfma_$x gpurun_out/mfma_$x.json --label $x; done
exit $rc
