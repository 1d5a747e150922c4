mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread -k "sliced or bench_route or batched_graphs" > gpurun_out/r05f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05f_tests.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python tools/ab_flags.py --configs ns --batch 64 --flags 0 > gpurun_out/r05f_ab_b64_new.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab_flags.py --configs ns --batch 64 --flags 0 --lib tools/ab/libgll_r04.so > gpurun_out/r05f_ab_b64_r04.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ab_flags.py --configs ns --batch 64 --flags 0 > gpurun_out/r05f_ab_b64_new2.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 200 --cpu-seconds 0 > gpurun_out/r05f_bench.json 2>gpurun_out/r05f_bench.err || exit $?
