# Profile session (GPU box): rocprofv3 kernel stats of the shipped paths, PMC byte passes
# (FETCH_SIZE / WRITE_SIZE, separate runs) and the Gram's MFMA counters, for the configs the
# bench reports.  One naming scheme everywhere: <tag>_<cfg>_* with cfg in
#   ns, fullysup, stress (bench.py --config), ns_b64, fullysup_b64 (the batched entry, B = 64).
#   bash tools/prof_session.sh <tag> [cfg ...]   -> gpurun_out/<tag>_{prof,pmcf,pmcw,mfma}_<cfg>
# then, on the build side, `bash tools/collect_profiles.sh <tag>` copies the summaries into
# profiles/ as <tag>_<cfg>_kernel_stats.csv, <tag>_pmc_<cfg>.json, <tag>_mfma_<cfg>.json --
# the names bench.py cites (rocprof_stats, traffic, gram_mfma_pmc).
T=${1:-r05}
shift
CFGS=${*:-ns ns_b64 fullysup fullysup_b64 stress}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && R=$PWD
P="rocprofv3"
cmd_for() {   # the workload of a cfg: the bench's single-graph step, or the batched probe
  case $1 in
    ns|fullysup) echo "python3 $R/bench.py --config $1 --steps 60 --warmup 10 --cpu-seconds 0 --no-profile --batch 0";;
    stress) echo "python3 $R/bench.py --config stress --steps 10 --warmup 3 --cpu-seconds 0 --no-profile --batch 0";;
    ns_b64) echo "PROBE_B=64 PROBE_CFG=ns python3 $R/tools/batch_probe.py";;
    fullysup_b64) echo "PROBE_B=64 PROBE_CFG=fullysup python3 $R/tools/batch_probe.py";;
    stress_b64) echo "PROBE_B=64 PROBE_CFG=stress PROBE_EPS=auto python3 $R/tools/batch_probe.py";;
  esac
}
MF="--pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv"
ST_ARGS="--kernel-trace --stats --output-format csv"
steps=()
for cfg in $CFGS; do
  C=$(cmd_for $cfg)
  # (environment assignments go before rocprofv3, never between it and the program)
  env_part=${C%%python3*}; prog=${C#"$env_part"}
  steps+=("${T}_prof_${cfg}:180:$env_part $P $ST_ARGS -d gpurun_out/${T}_prof_${cfg} -o run -- $prog")
  steps+=("${T}_pmcf_${cfg}:150:$env_part $P --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_pmcf_${cfg} -o run -- $prog")
  steps+=("${T}_pmcw_${cfg}:150:$env_part $P --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_pmcw_${cfg} -o run -- $prog")
  case $cfg in ns|ns_b64|stress) steps+=("${T}_mfma_${cfg}:150:$env_part $P $MF -d gpurun_out/${T}_mfma_${cfg} -o run -- $prog");; esac
done
# the build identity these summaries belong to (bench.py cites a summary only for its own build)
python3 -c "import json, time; from graphlearninglayer_amd import _lib; \
json.dump({'build_id': _lib.build_id(), 'recorded': time.strftime('%Y-%m-%dT%H:%M:%S'), \
'tag': '$T'}, open('gpurun_out/${T}_build.json', 'w'))"
bash tools/gpu_steps.sh "${steps[@]}"
rc=$?
for cfg in $CFGS; do
  [[ -d gpurun_out/${T}_pmcf_$cfg && -d gpurun_out/${T}_pmcw_$cfg ]] && \
    python3 tools/pmc_summary.py gpurun_out/${T}_pmcf_$cfg gpurun_out/${T}_pmcw_$cfg gpurun_out/${T}_pmc_$cfg.json --config $cfg
  [[ -d gpurun_out/${T}_mfma_$cfg ]] && python3 tools/mfma_summary.py gpurun_out/${T}_mfma_$cfg gpurun_out/${T}_mfma_$cfg.json --label $cfg
done
exit $rc
