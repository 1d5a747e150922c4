# r05zf: upper bound of balancing the fused gradient: rows cut to 16 edges (timing only)
cd "$GRAFT_REPO_ROOT"
A="python3 tools/ab_flags.py --flags 0 --reps 10 --configs ns --batch 1"
bash tools/gpu_steps.sh "r05zf_ab_new:200:$A" "r05zf_ab_trunc:200:$A --lib tools/libgll_alt_trunc.so" \
  "r05zf_ab_new2:200:$A" "r05zf_ab_trunc2:200:$A --lib tools/libgll_alt_trunc.so"
