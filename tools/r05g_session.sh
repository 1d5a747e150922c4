mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r05g_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05g_tests.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05g_smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r05g_bench.json 2>gpurun_out/r05g_bench.err || exit $?
