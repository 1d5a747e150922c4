# round-4 GPU session s: the Gram tail's subtiles over k-slices; order_perm batched -- tests, stress A/B
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04s_tests:400:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k 'tail or gram or locality or stress or fixture'" \
  "r04s_ab_tail:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --knob 4 --values 0,2,1,0,2 --reps 10"
