# Final checks of a build on the GPU box: every GPU test, smoke, the default bench line
#   bash tools/final_check.sh <tag>   -> gpurun_out/<tag>_{tests,smoke,bench}.log, <tag>_bench.json
T=${1:-final}
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "${T}_tests:900:python3 -u -m pytest -q --timeout 150 --timeout-method thread tests -m gpu" \
  "${T}_smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "${T}_bench:400:python3 bench.py > gpurun_out/${T}_bench.json"
