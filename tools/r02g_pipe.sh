#!/bin/bash
# Round-2g session (GPU box): batched build pipeline A/B (GLL_PIPE_CHUNKS 1/2/4 at NS, FullySup
# and stress B = 64 / 8), then the GPU tests.  The pipeline and its GLL_PIPE_CHUNKS switch were
# removed after this measurement (slower at every chunk count); kept as the record.  Every GPU step has its own limit; any failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
set -o pipefail
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 6 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  [[ $rc == 0 ]] || exit $rc
}
for nc in ${CHUNKS:-1 2 4}; do
  GLL_PIPE_CHUNKS=$nc PROBE_B=64 run "pipe_ns_$nc" 180 python tools/batch_probe.py
done
for nc in ${CHUNKS:-1 2 4}; do
  GLL_PIPE_CHUNKS=$nc PROBE_B=64 PROBE_CFG=fullysup run "pipe_fs_$nc" 180 python tools/batch_probe.py
done
[[ -n $NO_TESTS ]] || run tests 900 python -u -m pytest tests -m gpu -v -rf -x --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
exit 0
