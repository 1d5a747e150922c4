# r06w (part 2): the whole GPU suite again (d = 2 case), profile session for fullysup_b64,
# stress, stress_b64, then the bench lines that cite the r06w profiles
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r06w_gpu_tests:420:python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread"
rc=$?
[ $rc -ge 124 ] && exit $rc
bash tools/prof_session.sh r06w fullysup_b64 stress stress_b64 || exit $?
bash tools/collect_profiles.sh r06w > /dev/null 2>&1 || true
mkdir -p gpurun_out/r06w_profiles && cp profiles/r06w_* gpurun_out/r06w_profiles/ 2>/dev/null
bash tools/gpu_steps.sh \
  "r06w_bench_ns:400:python3 bench.py > gpurun_out/r06w_bench_ns.json" \
  "r06w_bench_fullysup:400:python3 bench.py --config fullysup > gpurun_out/r06w_bench_fullysup.json" \
  "r06w_bench_stress:500:python3 bench.py --config stress --steps 20 --warmup 5 > gpurun_out/r06w_bench_stress.json"
