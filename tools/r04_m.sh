# round-4 GPU session m: the Gram's short last round as 128-subtiles -- tile tests, A/B
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04m_tests:300:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k 'gram or locality or stress_fixture or fixture'" \
  "r04m_ab_tail:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --knob 4 --values 0,1,0,1 --reps 10 && python3 tools/ab_flags.py --configs ns --batch 64 --flags 0 --knob 4 --values 0,1,0,1 --reps 20"
