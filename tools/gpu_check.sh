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
[[ $STEPS == *tests* ]] && run tests 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-}
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps ${BENCH_STEPS:-200} --warmup 20 ${BENCH_ARGS:-}
exit 0
