# round-4 GPU session f: a shared status sink no longer takes one atomic per CG column
# workgroup of a batch -- A/B with and without a sink, bench, batched tests
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04f_ab_sink:200:python3 tools/ab_flags.py --configs ns --batch 64 --flags 0 --reps 30 && python3 tools/ab_flags.py --configs ns --batch 64 --flags 0 --reps 30 --sink" \
  "r04f_tests:300:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k 'batched or status or nonconv or warn'" \
  "r04f_bench:300:python3 bench.py --cpu-seconds 0 > gpurun_out/r04f_bench.json"
