# per-column CG: Neumann-preconditioned (MODE 3) vs Jacobi (MODE 1) single-reduction, twice
for rep in 1 2; do
for v in 3 1; do
  echo "== MODE=$v rep $rep"
  GLL_CG_MODE=$v python -u tools/ab_flags.py --flags 0 --configs ns,plumbing --batch 1,64 --reps 100 2>&1 | grep -v amdgpu.ids || exit $?
done; done
echo "== default"
python -u tools/ab_flags.py --flags 0,16384 --configs ns --batch 1 --reps 300 2>&1 | grep -v amdgpu.ids
