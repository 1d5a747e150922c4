#!/bin/bash
# Round-2g session (GPU box): whole-row gradient with the register-form coefficient vs the
# generic per-class loop (GLL_GRAD_CV=0) at NS and FullySup, B = 1 and 64; the utils.laplace
# probe at the reference's size; then the GPU tests.  Each GPU step has its own limit; any
# failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "^B=|^n=|passed|failed|Error" "gpurun_out/$name.log" | tail -n 8
  echo "=== $name rc=$rc"
  [[ $rc == 0 ]] || exit $rc
}
for cv in 0 1; do
  GLL_GRAD_CV=$cv PROBE_B=1,64 run "grad_ns_cv$cv" 180 python tools/batch_probe.py
  GLL_GRAD_CV=$cv PROBE_B=1 PROBE_CFG=fullysup run "grad_fs_cv$cv" 180 python tools/batch_probe.py
done
[[ -n $NO_LAPLACE ]] || run laplace 300 python tools/laplace_probe.py
[[ -n $NO_TESTS ]] || run tests 900 python -u -m pytest tests -m gpu -v -rf -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
[[ -n $NO_SMOKE ]] || run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
exit 0
