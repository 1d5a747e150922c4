# round-4 GPU session q: select (second row read skipped when lists are complete, x_i by
# LDS-DMA, 8-wave form A/B); two-row ELL CG in MODE 1 -- full GPU suite, A/B, stress trace
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04q_tests:600:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu" \
  "r04q_ab_sel:400:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --knob 3 --values 0,3,0,3 --reps 10 && python3 tools/ab_flags.py --configs ns,fullysup --batch 64 --flags 0 --knob 3 --values 0,3,0,3 --reps 10" \
  "r04q_trace_stress:150:TRACE_CFG=stress python3 tools/trace_probe.py"
