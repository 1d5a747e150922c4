# r06zf (part 2): profile session for fullysup_b64, stress, stress_b64, then the bench lines
# that cite the r06zf profiles
cd "$GRAFT_REPO_ROOT"
bash tools/prof_session.sh r06zf fullysup_b64 stress stress_b64 || exit $?
bash tools/collect_profiles.sh r06zf > /dev/null 2>&1 || true
mkdir -p gpurun_out/r06zf_profiles && cp profiles/r06zf_* gpurun_out/r06zf_profiles/ 2>/dev/null
bash tools/gpu_steps.sh \
  "r06zf_bench_ns:400:python3 bench.py > gpurun_out/r06zf_bench_ns.json" \
  "r06zf_bench_fullysup:400:python3 bench.py --config fullysup > gpurun_out/r06zf_bench_fullysup.json" \
  "r06zf_bench_stress:500:python3 bench.py --config stress --steps 20 --warmup 5 > gpurun_out/r06zf_bench_stress.json"
