# round-4 GPU session c: sampled traces (stress select, B = 64 CG), the locality-order A/B and
# the batched CG geometry A/B
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04c_trace_stress:150:TRACE_CFG=stress python3 tools/trace_probe.py" \
  "r04c_trace_b64:120:TRACE_B=64 python3 tools/trace_probe.py" \
  "r04c_ab_order:200:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0,262144,0,262144 --reps 10" \
  "r04c_ab_geom:300:python3 tools/ab_flags.py --configs ns --batch 64 --flags 0 --geoms 0,1,2,3,4,5,6,7,8,9,0 --reps 30" \
  "r04c_test_geom:200:python3 -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k 'geometry_variants or bench_route'"
