# round-4 GPU session b: CG traces (timestamp build) at B = 64 and B = 1, then the profile session
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04b_trace_b64:120:TRACE_B=64 python3 tools/trace_probe.py" \
  "r04b_trace_b1:120:TRACE_B=1 python3 tools/trace_probe.py" || exit $?
bash tools/r04_prof.sh r04b
