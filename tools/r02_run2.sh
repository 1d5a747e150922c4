cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
STEPS=tests bash tools/gpu_check.sh && \
timeout -k 10 300 python bench.py --config stress --steps 20 --warmup 3 --cpu-seconds 0 --batch 0 > gpurun_out/bench_stress.log 2>&1 && tail -1 gpurun_out/bench_stress.log | cut -c1-1500 && \
timeout -k 10 300 python bench.py --config fullysup --steps 100 --warmup 10 --cpu-seconds 0 --batch 0 > gpurun_out/bench_fullysup.log 2>&1 && tail -1 gpurun_out/bench_fullysup.log | cut -c1-1500 && \
timeout -k 10 120 python tools/base_loader_probe.py > gpurun_out/base_loader.log 2>&1; cat gpurun_out/base_loader.log
