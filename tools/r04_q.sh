# round-4 GPU session q: select without the second row read when the lane lists are complete;
# two-row ELL CG in MODE 1 -- full GPU suite, stress A/B + trace
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04q_tests:600:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu" \
  "r04q_ab_stress:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --reps 10" \
  "r04q_trace_stress:150:TRACE_CFG=stress python3 tools/trace_probe.py"
