# r06k (part 2): profile session for fullysup_b64, stress, stress_b64 (same build, tag r06k), then
# the bench lines of the shipped build citing them
cd "$GRAFT_REPO_ROOT"
bash tools/prof_session.sh r06k fullysup_b64 stress stress_b64
rc=$?
[ $rc -ge 124 ] && exit $rc
bash tools/collect_profiles.sh r06k > /dev/null 2>&1 || true
mkdir -p gpurun_out/r06k_profiles && cp profiles/r06k_* gpurun_out/r06k_profiles/ 2>/dev/null
bash tools/gpu_steps.sh \
  "r06k_bench_ns:400:python3 bench.py > gpurun_out/r06k_bench_ns.json" \
  "r06k_bench_fullysup:400:python3 bench.py --config fullysup > gpurun_out/r06k_bench_fullysup.json" \
  "r06k_bench_stress:500:python3 bench.py --config stress --steps 20 --warmup 5 > gpurun_out/r06k_bench_stress.json"
