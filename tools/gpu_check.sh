#!/bin/bash
# Guarded GPU session: every GPU step has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HIP_LAUNCH_BLOCKING=${HIP_LAUNCH_BLOCKING:-0}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 25 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  case $rc in 0|1) return 0;; *) echo "fatal rc=$rc in $name; stopping"; exit $rc;; esac
}
STEPS=${STEPS:-smoke,tests,bench}
[[ $STEPS == *info* ]] && run info 60 bash -c "rocminfo | grep -E 'Marketing|gfx|Compute Unit' | head -8; nproc; lscpu | grep 'Model name'"
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *tests* ]] && run tests 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps ${BENCH_STEPS:-200} --warmup 20 ${BENCH_ARGS:-}
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  R=$PWD
  PROF_CFG=${PROF_CFG:-ns}
  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$PROF_CFG" -o run -- \
      python3 "$R/bench.py" --config $PROF_CFG --steps ${PROF_STEPS:-100} --warmup 10 --cpu-seconds 0 --no-profile
  find "$R/gpurun_out/prof_$PROF_CFG" -name '*kernel_stats.csv' -exec cat {} \; | head -30
fi
if [[ $STEPS == *pmc* ]]; then
  export TMPDIR=/tmp
  R=$PWD
  PROF_CFG=${PROF_CFG:-ns}
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_fetch_$PROF_CFG" -o run -- \
      python3 "$R/bench.py" --config $PROF_CFG --steps 20 --warmup 5 --cpu-seconds 0 --no-profile
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_write_$PROF_CFG" -o run -- \
      python3 "$R/bench.py" --config $PROF_CFG --steps 20 --warmup 5 --cpu-seconds 0 --no-profile
fi
if [[ $STEPS == *scale* ]]; then
  run scale 600 python tools/scale_probe.py
fi
if [[ $STEPS == *host* ]]; then
  run host 300 python tools/host_overhead.py
fi
if [[ $STEPS == *mfmalist* ]]; then
  run counters_list 120 rocprofv3 -L
  grep -oE "(SQ_[A-Z_]*MFMA[A-Z0-9_]*|GRBM_GUI_ACTIVE|SQ_BUSY_CYCLES|SQ_WAVE_CYCLES)" gpurun_out/counters_list.log | sort -u | head -40
fi
if [[ $STEPS == *ctr* ]]; then
  export TMPDIR=/tmp
  R=$PWD
  run counters_list 120 rocprofv3 -L
  grep -oE "(GRBM_GUI_ACTIVE|SQ_WAVES|SQ_BUSY_CYCLES|SQ_WAIT_INST_ANY|SQ_WAIT_ANY|SQ_ACTIVE_INST_ANY|SQ_INSTS_VALU|SQ_INSTS_MFMA|SQ_VALU_MFMA_BUSY_CYCLES|SQ_INSTS_VALU_MFMA_MOPS_F32|SQ_WAVE_CYCLES|TA_BUSY_avr|SQ_INSTS_LDS|SQ_LDS_BANK_CONFLICT|SQ_INST_CYCLES_VMEM)[A-Za-z0-9_]*" gpurun_out/counters_list.log | sort -u | head -40
  run pmc_a 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_a" -o run -- \
      python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-seconds 0 --no-profile
  run pmc_b 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_b" -o run -- \
      python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-seconds 0 --no-profile
fi
exit 0
