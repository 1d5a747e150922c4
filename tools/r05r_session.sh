# r05r: two-phase ELL loads in the batched CG (tools/libgll_alt_head.so = the previous build)
cd "$GRAFT_REPO_ROOT"
A="python3 tools/ab_flags.py --configs ns --batch 64 --flags 0 --reps 10"
bash tools/gpu_steps.sh \
  "r05r_tests:200:python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread -k 'batched or bench_route or two_row'" \
  "r05r_ab_new:200:$A" "r05r_ab_head:200:$A --lib tools/libgll_alt_head.so" "r05r_ab_new2:200:$A" \
  "r05r_ab_head2:200:$A --lib tools/libgll_alt_head.so"
