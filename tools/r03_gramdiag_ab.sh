# gram_pk2_kernel epilogue: LDS-staged direct rows (GLL_GRAM_DIAG=0, default), per-element stores
# (=2, the round-2 epilogue), none (=1: no D2 stores, timing only), twice each.
for rep in 1 2; do
for v in "GLL_GRAM_DIAG=0" "GLL_GRAM_DIAG=2" "GLL_GRAM_DIAG=1"; do
  echo "== $v rep $rep"
  env $v python -u tools/ab_flags.py --flags 0 --configs ns --batch 64 --reps 20 2>&1 | grep -v amdgpu.ids || exit $?
  env $v python -u tools/ab_flags.py --flags 0 --configs stress --batch 1 --reps 10 2>&1 | grep -v amdgpu.ids || exit $?
done; done
