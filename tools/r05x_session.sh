# r05x: RCAP 8(K-1)+8, unrolled row sort, hub label batches; tools/libgll_alt_head.so = before
cd "$GRAFT_REPO_ROOT"
A="python3 tools/ab_flags.py --batch 1 --flags 0 --reps 5"
bash tools/gpu_steps.sh \
  "r05x_tests:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k 'hub or stress or fixture or duplicate or batched_two_row or bench_route'" \
  "r05x_trace_stress:120:TRACE_CFG=stress TRACE_EPS=0 python tools/trace_probe.py" \
  "r05x_ab_new:300:$A --configs stress,ns,fullysup" "r05x_ab_head:300:$A --configs stress,ns,fullysup --lib tools/libgll_alt_head.so" \
  "r05x_ab_new2:300:$A --configs stress,ns,fullysup"
