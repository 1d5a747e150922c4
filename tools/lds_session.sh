# LDS counters per kernel (bank-conflict cycles vs all LDS-array cycles) for the CG configs.
#   bash tools/lds_session.sh <tag>  -> gpurun_out/<tag>_lds_<cfg>/ and <tag>_lds_<cfg>.txt
T=${1:-r05s}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && R=$PWD
PM="--pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv"
bash tools/gpu_steps.sh \
  "${T}_lds_ns_b64:150:PROBE_B=64 PROBE_CFG=ns rocprofv3 $PM -d gpurun_out/${T}_lds_ns_b64 -o run -- python3 $R/tools/batch_probe.py" \
  "${T}_lds_ns:150:rocprofv3 $PM -d gpurun_out/${T}_lds_ns -o run -- python3 $R/bench.py --config ns --steps 60 --warmup 10 --cpu-seconds 0 --no-profile --batch 0" \
  "${T}_lds_fullysup:150:rocprofv3 $PM -d gpurun_out/${T}_lds_fullysup -o run -- python3 $R/bench.py --config fullysup --steps 60 --warmup 10 --cpu-seconds 0 --no-profile --batch 0"
rc=$?
for c in ns_b64 ns fullysup; do
  [ -d gpurun_out/${T}_lds_$c ] && python3 tools/counter_summary.py gpurun_out/${T}_lds_$c > gpurun_out/${T}_lds_$c.txt
done
[ $rc -ge 124 ] && exit $rc
timeout -k 10 240 python3 tools/batch_probe.py > gpurun_out/${T}_batch_scaling_ns.txt 2>&1 || exit $?
PROBE_CFG=fullysup PROBE_B=1,8,64 timeout -k 10 240 python3 tools/batch_probe.py > gpurun_out/${T}_batch_scaling_fullysup.txt 2>&1 || exit $?
