# batched CG: lazy vs eager ELL prologue (twice each)
for rep in 1 2; do
for v in 1 0; do
  echo "== LAZY=$v rep $rep"
  GLL_CG_LAZY=$v python -u tools/ab_flags.py --flags 0 --configs ns,fullysup --batch 64 --reps 30 2>&1 | grep -v amdgpu.ids || exit $?
done; done
