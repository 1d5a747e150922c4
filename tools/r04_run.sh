# round-4 GPU session: launch costs, host breakdown, bench, targeted GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tools/csrc/launch_probe > gpurun_out/r04a_launch.txt 2>&1 || exit 1
timeout -k 10 300 python tools/host_breakdown.py > gpurun_out/r04a_host.txt 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || exit 3
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_callers.py > gpurun_out/r04a_tests.txt 2>&1 || exit 4
