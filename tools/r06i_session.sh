# r06i: the batched adjoint's Chebyshev iteration (single direction buffer, the forward's Ritz
# interval) and the Gram tail as 64-subtiles -- GPU tests, A/B (GLL_KNOB_CHEB 0/1, GLL_KNOB_GRAM_TAIL
# 0/2/1, the previous build alt/libgll_head.so), rocprof kernel stats of B = 64 NS and stress
cd "$GRAFT_REPO_ROOT"
R=$PWD
bash tools/gpu_steps.sh \
  "r06i_tests:500:python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k 'chebyshev or batched or bench_route or gram or stress'" \
  "r06i_ab_cheb:300:python3 tools/ab_flags.py --configs ns --batch 64 --knob 6 --values 0,1 --reps 30 && python3 tools/ab_flags.py --configs ns --batch 64 --reps 30 --lib alt/libgll_head.so" \
  "r06i_ab_tail:400:python3 tools/ab_flags.py --configs stress --batch 1 --knob 4 --values 0,2,1 --reps 10 && python3 tools/ab_flags.py --configs ns,fullysup --batch 64 --knob 4 --values 0,1 --reps 20" \
  "r06i_prof_ns_b64:200:PROBE_B=64 PROBE_CFG=ns rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06i_prof_ns_b64 -o run -- python3 $R/tools/batch_probe.py" \
  "r06i_prof_stress:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06i_prof_stress -o run -- python3 $R/bench.py --config stress --steps 10 --warmup 3 --cpu-seconds 0 --no-profile --batch 0"
