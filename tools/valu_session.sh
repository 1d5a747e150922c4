# Issue counters per kernel (VALU / SALU / LDS instructions and active cycles vs wave cycles)
#   bash tools/valu_session.sh <tag>  -> gpurun_out/<tag>_valu_<cfg>.txt
T=${1:-r05v}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && R=$PWD
PM="--pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv"
bash tools/gpu_steps.sh \
  "${T}_valu_ns_b64:150:PROBE_B=64 PROBE_CFG=ns rocprofv3 $PM -d gpurun_out/${T}_valu_ns_b64 -o run -- python3 $R/tools/batch_probe.py" \
  "${T}_valu_stress:150:rocprofv3 $PM -d gpurun_out/${T}_valu_stress -o run -- python3 $R/bench.py --config stress --steps 10 --warmup 3 --cpu-seconds 0 --no-profile --batch 0"
rc=$?
for c in ns_b64 stress; do
  [ -d gpurun_out/${T}_valu_$c ] && python3 tools/counter_summary.py gpurun_out/${T}_valu_$c > gpurun_out/${T}_valu_$c.txt
done
[ $rc -ge 124 ] && exit $rc
exit 0
