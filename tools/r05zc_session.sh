# r05zc: fused backward stages neighbour rows in LDS during the wait; alt_head = before
cd "$GRAFT_REPO_ROOT"
A="python3 tools/ab_flags.py --flags 0 --reps 10 --configs ns --batch 1"
bash tools/gpu_steps.sh \
  "r05zc_tests:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_callers.py -m gpu -q --timeout 200 --timeout-method thread -k 'fused or fixture or deterministic or ns or class or hub'" \
  "r05zc_trace:120:TRACE_CFG=ns python tools/trace_probe.py > gpurun_out/r05zc_trace_ns.txt" \
  "r05zc_ab_new:200:$A" "r05zc_ab_head:200:$A --lib tools/libgll_alt_head.so" "r05zc_ab_new2:200:$A" "r05zc_ab_head2:200:$A --lib tools/libgll_alt_head.so"
