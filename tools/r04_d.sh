# round-4 GPU session d: the select without per-lane key lists (threshold scan for every list
# size, full-row fallback) and the occupancy form for large single graphs -- full GPU suite,
# then the select form / locality order A/B at stress and the other configs' timings
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04d_tests:600:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu" \
  "r04d_ab_stress:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0,262144 --knob 3 --values 1,2,0 --reps 10" \
  "r04d_ab_other:300:python3 tools/ab_flags.py --configs ns,fullysup --batch 1,64 --flags 0 --reps 30"
