# round-4 GPU session o: order kernels without global atomics -- locality tests, stress A/B, stress rocprof
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "r04o_tests:300:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k 'locality or stress'" \
  "r04o_ab_stress:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0,262144 --reps 10" \
  "r04o_prof_stress:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04o_prof_stress -o run -- python3 bench.py --config stress --steps 10 --warmup 3 --cpu-seconds 0 --no-profile --batch 0"
