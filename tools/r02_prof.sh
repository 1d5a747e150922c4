# Round-2 profile session (GPU box): MFMA counters for the Gram at NS / B=64 / stress,
# rocprof stats + FETCH/WRITE for the B=64 batched run and for stress.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && R=$PWD
P="timeout -s KILL 120 rocprofv3"
MF="--pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv"
NS="python3 $R/bench.py --config ns --steps 30 --warmup 5 --cpu-seconds 0 --no-profile --batch 0"
ST="python3 $R/bench.py --config stress --steps 10 --warmup 3 --cpu-seconds 0 --no-profile --batch 0"
B64="python3 $R/tools/batch_probe.py"
export PROBE_B=64
# (a --pmc pass over the whole stress call segfaulted at process exit inside the profiler once the
# whole-GPU CG went cooperative; the Gram's counters come from the graph-only probe instead, and
# every stress pass launches that CG as an ordinary launch, GLL_GRID_COOP=0: kernel-trace alone
# also segfaulted at exit with the cooperative launch)
GS="python3 $R/tools/graph_probe.py"
[[ ${SKIP_DONE:-0} -ge 1 ]] || { $P $MF -d $R/gpurun_out/mfma_ns -o run -- $NS > gpurun_out/mfma_ns.log 2>&1 && \
$P $MF -d $R/gpurun_out/mfma_b64 -o run -- $B64 > gpurun_out/mfma_b64.log 2>&1; } && \
[[ ${SKIP_DONE:-0} == 2 ]] || { PROBE_CFG=stress $P $MF -d $R/gpurun_out/mfma_stress -o run -- $GS > gpurun_out/mfma_stress.log 2>&1 && \
$P --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b64 -o run -- $B64 > gpurun_out/prof_b64.log 2>&1 && \
$P --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_b64 -o run -- $B64 > gpurun_out/pmc_fetch_b64.log 2>&1 && \
$P --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_b64 -o run -- $B64 > gpurun_out/pmc_write_b64.log 2>&1; } && \
GLL_GRID_COOP=0 $P --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stress -o run -- $ST > gpurun_out/prof_stress.log 2>&1 && \
GLL_GRID_COOP=0 $P --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_stress -o run -- $ST > gpurun_out/pmc_fetch_stress.log 2>&1 && \
GLL_GRID_COOP=0 $P --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_stress -o run -- $ST > gpurun_out/pmc_write_stress.log 2>&1
rc=$?
echo "profile session rc=$rc"
for x in ns b64 stress; do [[ -d gpurun_out/mfma_$x ]] && python3 tools/mfma_summary.py gpurun_out/mfma_$x gpurun_out/mfma_$x.json --label $x; done
exit $rc
