# Batched CG: column pairs / quads (cg_ell2_kernel) against the one-column kernel, twice each.
for rep in 1 2; do
for v in "GLL_CG_NC=1" "GLL_CG_NC=2" "GLL_CG_NC=4" "GLL_CG_NC=2 GLL_CG_NT=512" "GLL_CG_NC=4 GLL_CG_NT=512"; do
  echo "== $v rep $rep"
  env $v python -u tools/ab_flags.py --flags 0 --configs ns --batch 8,64 --reps 30 2>&1 | grep -v amdgpu.ids || exit $?
done; done
