# round-4 GPU session e: the select's exact distances as an explicit fma chain (both select
# forms bitwise equal), full GPU suite, stress A/B of the select forms
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04e_tests:600:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu" \
  "r04e_ab_stress:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0,262144 --knob 3 --values 1,2,0 --reps 10" || [ $? -lt 124 ] && bash tools/gpu_steps.sh \
  "r04e_bench:300:python3 bench.py --cpu-seconds 0 > gpurun_out/r04e_bench.json" \
  "r04e_ab_b64:200:python3 tools/ab_flags.py --configs ns --batch 64 --flags 0 --reps 30"
