# round-4 GPU session p: whole-GPU CG with 8 gathers per lane per round (trace, A/B, tests); the
# two-row register-ELL CG of single graphs (1024 < m <= 2048) in MODE 3 (main) vs MODE 1 (alt)
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04p_gv_trace:120:python3 tools/gv_trace.py" \
  "r04p_ab_stress:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --reps 10" \
  "r04p_ab_ell2:200:python3 tools/ab_flags.py --configs fullysup --batch 1 --flags 512 --reps 20 && python3 tools/ab_flags.py --configs fullysup --batch 1 --flags 512 --reps 20 --lib tools/libgll_alt.so && python3 tools/ab_flags.py --configs fullysup --batch 1 --flags 512 --reps 20" \
  "r04p_trace_stress:150:TRACE_CFG=stress python3 tools/trace_probe.py" \
  "r04p_tests:300:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k 'grid or laplace or stress or locality or balanced or fullysup'"
