# batched NS CG: ELL width and workgroups per CU (LDS padding) A/B, twice each
for rep in 1 2; do
for v in "12 0" "24 0" "12 40000" "12 54000" "12 80000"; do set -- $v
  echo "== BS=$1 LDS_PAD=$2 rep $rep"
  GLL_CG_BS=$1 GLL_CG_LDS_PAD=$2 python -u tools/ab_flags.py --flags 0 --configs ns --batch 64 --reps 30 2>&1 | grep -v amdgpu.ids || exit $?
done; done
