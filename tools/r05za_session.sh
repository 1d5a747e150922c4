# r05za: row build -- forward match by LDS scan, prefetched-label RHS 16 per step; alt_head = before
cd "$GRAFT_REPO_ROOT"
A="python3 tools/ab_flags.py --flags 0 --reps 5"
bash tools/gpu_steps.sh \
  "r05za_tests:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k 'hub or stress or fixture or duplicate or batched or bench_route or deterministic'" \
  "r05za_trace:200:TRACE_CFG=stress TRACE_EPS=0 python tools/trace_probe.py > gpurun_out/r05za_trace_stress.txt && TRACE_CFG=ns python tools/trace_probe.py > gpurun_out/r05za_trace_ns.txt" \
  "r05za_ab_new:300:$A --configs stress,ns,fullysup --batch 1 && $A --configs ns,fullysup --batch 64" \
  "r05za_ab_head:300:$A --configs stress,ns,fullysup --batch 1 --lib tools/libgll_alt_head.so && $A --configs ns,fullysup --batch 64 --lib tools/libgll_alt_head.so" \
  "r05za_ab_new2:300:$A --configs stress,ns,fullysup --batch 1 && $A --configs ns,fullysup --batch 64"
