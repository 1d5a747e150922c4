# fp16 x 2^e distance storage (default for batches on the pre-split route) against fp32
# (GLL_D2_F32=1), and the fragment-pipelined 256-tile GEMM (GLL_GRAM_PIPE=1); single graphs
# (stress) with GLL_D2_HALF1=1 against their fp32 default. Twice each.
for rep in 1 2; do
for v in "GLL_D2_F32=0" "GLL_D2_F32=1" "GLL_GRAM_PIPE=1"; do
  echo "== $v rep $rep"
  env $v python -u tools/ab_flags.py --flags 0 --configs ns,fullysup --batch 64 --reps 20 2>&1 | grep -v amdgpu.ids || exit $?
done
for v in "GLL_D2_HALF1=0" "GLL_D2_HALF1=1" "GLL_GRAM_PIPE=1"; do
  echo "== $v rep $rep"
  env $v python -u tools/ab_flags.py --flags 0 --configs stress --batch 1 --reps 10 2>&1 | grep -v amdgpu.ids || exit $?
done; done
