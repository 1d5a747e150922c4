# round-4 GPU session w: bench with the event pool filled before the timed regions; smoke
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04w_bench:400:python3 bench.py > gpurun_out/r04w_bench.json" \
  "r04w_smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'"
