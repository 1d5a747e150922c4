#!/bin/bash
# Round-2g session (GPU box): batch probe at NS / FullySup (B = 1, 64), the GPU tests, smoke and
# the default bench line.  Each GPU step has its own limit; any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
TAG=${TAG:-r02g}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "^B=|^n=|passed|failed|Error|\"metric\"" "gpurun_out/$name.log" | cut -c1-400 | tail -n 8
  echo "=== $name rc=$rc"
  [[ $rc == 0 ]] || exit $rc
}
PROBE_B=1,64 run "${TAG}_probe_ns" 180 python tools/batch_probe.py
PROBE_B=1,64 PROBE_CFG=fullysup run "${TAG}_probe_fs" 180 python tools/batch_probe.py
[[ -n $NO_TESTS ]] || run "${TAG}_tests" 900 python -u -m pytest tests -m gpu -v -rf -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
[[ -n $NO_SMOKE ]] || run "${TAG}_smoke" 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ -n $NO_BENCH ]] || run "${TAG}_bench" 600 python bench.py
exit 0
