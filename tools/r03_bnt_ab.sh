# Batched per-column CG geometry: 256 x 2 (MODE 1, default) against 512 x 1 (MODE 3 / MODE 1), twice each.
for rep in 1 2; do
for v in "GLL_CG_BNT=0" "GLL_CG_BNT=512" "GLL_CG_BNT=512 GLL_CG_MODE=1"; do
  echo "== $v rep $rep"
  env $v python -u tools/ab_flags.py --flags 0 --configs ns --batch 8,64 --reps 30 2>&1 | grep -v amdgpu.ids || exit $?
done; done
