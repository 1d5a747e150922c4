# round-4 GPU session l: whole-GPU CG step sizes per wave (no broadcast barriers) -- grid tests,
# iteration trace, stress A/B
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04l_tests:300:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k 'grid or stress or laplace or rescue or locality'" \
  "r04l_gv_trace:120:python3 tools/gv_trace.py" \
  "r04l_ab_stress:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --reps 10"
