# Pre-split Gram route: fp16 x 2^e distance storage (default) against fp32 (GLL_D2_F32=1), twice each.
for rep in 1 2; do
for v in "GLL_D2_F32=0" "GLL_D2_F32=1"; do
  echo "== $v rep $rep"
  env $v python -u tools/ab_flags.py --flags 0 --configs ns,fullysup --batch 64 --reps 20 2>&1 | grep -v amdgpu.ids || exit $?
  env $v python -u tools/ab_flags.py --flags 0 --configs stress --batch 1 --reps 10 2>&1 | grep -v amdgpu.ids || exit $?
done; done
