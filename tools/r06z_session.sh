# r06z: profiles of the shipped round-6 build (kernel stats, PMC bytes, MFMA counters) for every
# config the bench reports, then the bench lines that cite them
cd "$GRAFT_REPO_ROOT"
bash tools/prof_session.sh r06z ns ns_b64 fullysup fullysup_b64 stress stress_b64
for f in gpurun_out/r06z_prof_*; do :; done
bash tools/collect_profiles.sh r06z > /dev/null 2>&1 || true
mkdir -p gpurun_out/r06z_profiles && cp profiles/r06z_* gpurun_out/r06z_profiles/ 2>/dev/null
bash tools/gpu_steps.sh \
  "r06z_bench_ns:400:python3 bench.py > gpurun_out/r06z_bench_ns.json" \
  "r06z_bench_fullysup:400:python3 bench.py --config fullysup > gpurun_out/r06z_bench_fullysup.json" \
  "r06z_bench_stress:500:python3 bench.py --config stress --steps 20 --warmup 5 > gpurun_out/r06z_bench_stress.json"
