# r06o: packed-FP32 exact distances in the kNN select (v_pk_add_f32 / v_pk_fma_f32, two features
# per instruction) -- kNN / parity GPU tests, A/B against the previous build (alt/libgll_head.so)
# at every config, alternating builds; then the Gram tile-size A/B that r06n could not run
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r06o_tests:400:python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k 'select or knn or reference or stress or wide or batched_graphs'" \
  "r06o_ab:500:for i in 1 2; do python3 tools/ab_flags.py --configs ns,fullysup --batch 1,64 --reps 20 && python3 tools/ab_flags.py --configs ns,fullysup --batch 1,64 --reps 20 --lib alt/libgll_head.so; done" \
  "r06o_ab_stress:300:python3 tools/ab_flags.py --configs stress --batch 1 --reps 10 && python3 tools/ab_flags.py --configs stress --batch 1 --reps 10 --lib alt/libgll_head.so" \
  "r06o_ab_tile:300:python3 tools/ab_flags.py --configs ns --batch 64 --knob 2 --values 0,128 --reps 20"
