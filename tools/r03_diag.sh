# Abort diagnosis: smoke and the first batched test with HIP runtime error logging.
bash tools/r03_run.sh \
 "smoke_log:200:AMD_LOG_LEVEL=1 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "t_one:200:AMD_LOG_LEVEL=1 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k 'batched_graphs_equal_single_calls_bitwise and plumbing'"
