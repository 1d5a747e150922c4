# r05y: 256-tile Gram with 16-feature stages, three in flight; tools/libgll_alt_head.so = before
cd "$GRAFT_REPO_ROOT"
A="python3 tools/ab_flags.py --flags 0 --reps 5"
bash tools/gpu_steps.sh \
  "r05y_tests:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k 'tile or tail or batched or bench_route or stress or fp16'" \
  "r05y_ab_new:300:$A --configs stress --batch 1 && $A --configs ns --batch 64" \
  "r05y_ab_head:300:$A --configs stress --batch 1 --lib tools/libgll_alt_head.so && $A --configs ns --batch 64 --lib tools/libgll_alt_head.so" \
  "r05y_ab_new2:300:$A --configs stress --batch 1 && $A --configs ns --batch 64"
