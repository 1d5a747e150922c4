# r06d: FullySup shape, whole-GPU (grid) CG with 8-64 workgroups (GLL_KNOB_GRID_CAP) against the
# per-column balanced kernel (flags 0): nothing between 1 and ~78 workgroups was measured
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r06d_ab:400:python3 tools/ab_flags.py --flags 0 --reps 10 --configs fullysup --batch 1 && python3 tools/ab_flags.py --flags 1 --reps 10 --configs fullysup --batch 1 --knob 1 --values 0,8,16,24,32,48,64"
