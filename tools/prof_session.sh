# Round-4 profile session (GPU box): rocprofv3 kernel stats of the shipped paths, PMC byte
# passes (FETCH_SIZE / WRITE_SIZE, separate runs) and the Gram's MFMA counters.
#   bash tools/prof_session.sh <tag>     -> gpurun_out/<tag>_*  (copy the summaries to profiles/)
T=${1:-r04}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && R=$PWD
P="rocprofv3"
NS="python3 $R/bench.py --config ns --steps 60 --warmup 10 --cpu-seconds 0 --no-profile --batch 0"
ST="python3 $R/bench.py --config stress --steps 10 --warmup 3 --cpu-seconds 0 --no-profile --batch 0"
FS="python3 $R/bench.py --config fullysup --steps 60 --warmup 10 --cpu-seconds 0 --no-profile --batch 0"
MF="--pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv"
ST_ARGS="--kernel-trace --stats --output-format csv"
steps=()
for cfg in ns stress fullysup; do
  case $cfg in ns) C="$NS";; stress) C="$ST";; fullysup) C="$FS";; esac
  steps+=("${T}_prof_${cfg}:150:$P $ST_ARGS -d gpurun_out/${T}_prof_${cfg} -o run -- $C")
done
steps+=("${T}_prof_b64:150:PROBE_B=64 $P $ST_ARGS -d gpurun_out/${T}_prof_b64 -o run -- python3 $R/tools/batch_probe.py")
steps+=("${T}_prof_fs_b64:150:PROBE_B=64 PROBE_CFG=fullysup $P $ST_ARGS -d gpurun_out/${T}_prof_fs_b64 -o run -- python3 $R/tools/batch_probe.py")
for cfg in ns stress; do
  case $cfg in ns) C="$NS";; stress) C="$ST";; esac
  steps+=("${T}_pmcf_${cfg}:120:$P --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_pmcf_${cfg} -o run -- $C")
  steps+=("${T}_pmcw_${cfg}:120:$P --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_pmcw_${cfg} -o run -- $C")
done
steps+=("${T}_pmcf_b64:120:PROBE_B=64 $P --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_pmcf_b64 -o run -- python3 $R/tools/batch_probe.py")
steps+=("${T}_pmcw_b64:120:PROBE_B=64 $P --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_pmcw_b64 -o run -- python3 $R/tools/batch_probe.py")
steps+=("${T}_mfma_b64:120:PROBE_B=64 $P $MF -d gpurun_out/${T}_mfma_b64 -o run -- python3 $R/tools/batch_probe.py")
steps+=("${T}_mfma_stress:120:PROBE_CFG=stress $P $MF -d gpurun_out/${T}_mfma_stress -o run -- python3 $R/tools/graph_probe.py")
bash tools/gpu_steps.sh "${steps[@]}"
rc=$?
for cfg in ns stress b64; do
  [[ -d gpurun_out/${T}_pmcf_$cfg && -d gpurun_out/${T}_pmcw_$cfg ]] && \
    python3 tools/pmc_summary.py gpurun_out/${T}_pmcf_$cfg gpurun_out/${T}_pmcw_$cfg gpurun_out/${T}_pmc_$cfg.json --config $cfg
done
for x in b64 stress; do
  [[ -d gpurun_out/${T}_mfma_$x ]] && python3 tools/mfma_summary.py gpurun_out/${T}_mfma_$x gpurun_out/${T}_mfma_$x.json --label $x
done
exit $rc
