# GPU session helper: run steps in order, each under its own time limit; continue past
# an ordinary failure (rc 1: a failed test / probe assertion) but stop at once on a signal,
# abort, segfault or time limit (rc >= 124), so nothing more touches the GPU after a fault.
#   bash tools/gpu_steps.sh "<label>:<seconds>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
worst=0
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "== $label ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "== $label rc=$rc"; tail -n 5 "gpurun_out/$label.log"
  [[ $rc -gt $worst ]] && worst=$rc
  if [[ $rc -ge 124 || $rc -eq 134 || $rc -eq 139 ]]; then echo "stopping after $label"; exit $rc; fi
done
exit $worst
