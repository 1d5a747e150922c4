# One round-end GPU session (tag T, default r04): GPU suite, bench (headline + batched + auto-eps extra), A/B lines for
# the docs, and the profile set (rocprof stats + PMC + MFMA)
T=${1:-r04}
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "${T}_tests:600:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu" \
  "${T}_bench:400:python3 bench.py > gpurun_out/${T}_bench.json" \
  "${T}_ab:400:python3 tools/ab_flags.py --configs stress,fullysup,ns --batch 1 --flags 0 --reps 20 && python3 tools/ab_flags.py --configs ns,fullysup --batch 64 --flags 0 --reps 10" \
  || [ $? -lt 124 ] && bash tools/prof_session.sh $T
