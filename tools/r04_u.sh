# round-4 GPU session u: tail reduce through LDS slabs; nontemporal select D2 loads -- tests, A/B
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04u_tests:400:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k 'tail or gram or locality or stress or fixture or select or panel or duplicate'" \
  "r04u_ab_tail:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --knob 4 --values 0,2,0,2 --reps 10"
