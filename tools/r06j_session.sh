# r06j: the fused backward's class-ordered, XCD-local gradient rows -- GPU tests, A/B against the
# previous build (alt/libgll_head.so) at NS, and a profile session of NS (kernel stats, PMC bytes)
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r06j_tests:400:python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k 'fused or parity_against_reference or ns or gram_tail'" \
  "r06j_ab:300:for i in 1 2; do python3 tools/ab_flags.py --configs ns --batch 1 --reps 300 && python3 tools/ab_flags.py --configs ns --batch 1 --reps 300 --lib alt/libgll_head.so; done"
rc=$?
[ $rc -ge 124 ] && exit $rc
bash tools/prof_session.sh r06j ns
