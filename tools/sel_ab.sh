# Per-kernel timings across library variants (tools/variants/libgll_<V>.so swapped in place).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cp graphlearninglayer_amd/libgll.so /tmp/libgll_keep.so
for v in ${VARIANTS:-BASE}; do
  cp tools/variants/libgll_$v.so graphlearninglayer_amd/libgll.so
  timeout -k 10 300 python3 tools/ab_flags.py --flags 0 --configs ${CONFIGS:-ns,fullysup,stress} --batch ${BATCH:-1,64} --reps 20 2>&1 | grep flags | sed "s/^/$v /" || break
done
cp /tmp/libgll_keep.so graphlearninglayer_amd/libgll.so
