mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread -k "wide or sliced or bench_route or batched or fused or deterministic or parity_against or select_forms" > gpurun_out/r05e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05e_tests.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python bench.py --steps 100 --cpu-seconds 0 > gpurun_out/r05e_bench.json 2>gpurun_out/r05e_bench.err || exit $?
timeout -k 10 200 python tools/ab_flags.py --configs fullysup --batch 1 --flags 0,1 > gpurun_out/r05e_ab_fs_grid.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab_flags.py --configs ns --batch 64 --flags 0 > gpurun_out/r05e_ab_b64_new.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab_flags.py --configs ns --batch 64 --flags 0 --lib tools/ab/libgll_r04.so > gpurun_out/r05e_ab_b64_r04.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab_flags.py --configs ns --batch 64 --flags 0 > gpurun_out/r05e_ab_b64_new2.txt 2>&1 || exit $?
TRACE_CFG=stress timeout -k 10 120 python tools/trace_probe.py > gpurun_out/r05e_trace_stress.txt 2>&1 || exit $?
TRACE_B=64 timeout -k 10 120 python tools/trace_probe.py > gpurun_out/r05e_trace_b64.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab_flags.py --configs stress --batch 1 --flags 0 --knob 5 --values 0,2,1 --reps 20 > gpurun_out/r05e_ab_stress_pre.txt 2>&1 || exit $?
