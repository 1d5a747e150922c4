# r06c: fused backward with the long rows' neighbour rows LDS-DMA'd before the wait, against
# the build before it (tools/libgll_head.so.alt); fused-backward tests; the new tail profile
cd "$GRAFT_REPO_ROOT"
A="python3 tools/ab_flags.py --flags 0 --reps 20 --configs ns --batch 1"
bash tools/gpu_steps.sh \
  "r06c_tests:300:python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_callers.py -m gpu -q --timeout 200 --timeout-method thread -k 'fused or fixture or deterministic or ns or hub'" \
  "r06c_ab:300:echo head && $A --lib tools/libgll_head.so.alt && echo new && $A && echo head2 && $A --lib tools/libgll_head.so.alt && echo new2 && $A"
