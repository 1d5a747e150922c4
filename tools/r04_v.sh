# round-4 GPU session v: GPU suite, bench (headline + batched + auto-eps extra), A/B lines for
# the docs, and the profile set (rocprof stats + PMC + MFMA)
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04v_tests:600:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu" \
  "r04v_bench:400:python3 bench.py > gpurun_out/r04v_bench.json" \
  "r04v_ab:400:python3 tools/ab_flags.py --configs stress,fullysup,ns --batch 1 --flags 0 --reps 20 && python3 tools/ab_flags.py --configs ns,fullysup --batch 64 --flags 0 --reps 10" \
  || [ $? -lt 124 ] && bash tools/r04_prof.sh r04v
