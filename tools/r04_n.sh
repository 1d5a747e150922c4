# round-4 GPU session n: the Gram tail at stress (A/B), tile tests
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04n_ab_tail:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --knob 4 --values 0,1,0,1 --reps 10" \
  "r04n_tests:300:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k 'gram_256'"
