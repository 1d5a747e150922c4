# Round-3 final measurement session: rocprof stats / PMC / MFMA of the shipped paths, then the bench line.
bash tools/r03_prof.sh r03y; rc=$?
[[ $rc -ge 124 || $rc -eq 134 || $rc -eq 139 ]] && exit $rc
timeout -k 10 600 python bench.py --steps 200 --warmup 20 > gpurun_out/r03y_bench.log 2>&1; echo "bench rc=$?"; tail -c 600 gpurun_out/r03y_bench.log
