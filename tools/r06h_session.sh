# r06h: the batched adjoint's Chebyshev iteration -- GPU tests, A/B against the PCG adjoint
# (GLL_KNOB_CHEB = 1) and the previous build (alt/libgll_head.so), rocprof kernel stats of B = 64 NS
cd "$GRAFT_REPO_ROOT"
R=$PWD
bash tools/gpu_steps.sh \
  "r06h_tests:400:python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k 'chebyshev or batched or bench_route or fused_backward or balanced'" \
  "r06h_ab:300:python3 tools/ab_flags.py --configs ns --batch 64 --knob 6 --values 0,1 --reps 30 && python3 tools/ab_flags.py --configs ns --batch 64 --reps 30 --lib alt/libgll_head.so" \
  "r06h_prof_ns_b64:200:PROBE_B=64 PROBE_CFG=ns rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06h_prof_ns_b64 -o run -- python3 $R/tools/batch_probe.py"
