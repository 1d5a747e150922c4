mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python bench.py --cpu-seconds 0 --batch 0 > gpurun_out/r05h_bench_new$i.json 2>/dev/null || exit $?
timeout -k 10 200 python tools/ab/r04/bench.py --cpu-seconds 0 --batch 0 > gpurun_out/r05h_bench_r04_$i.json 2>/dev/null || exit $?
done
