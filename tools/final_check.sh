cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04f3_tests:600:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu" \
  "r04f3_smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "r04f3_bench:400:python3 bench.py > gpurun_out/r04f3_bench.json"
