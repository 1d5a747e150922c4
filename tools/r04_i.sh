# round-4 GPU session i: bench (headline + batched + auto-eps extra) and the profile set
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh "r04i_bench:400:python3 bench.py > gpurun_out/r04i_bench.json" \
  "r04i_ab_fs_ell:200:python3 tools/ab_flags.py --configs fullysup --batch 1 --flags 0,512 --reps 20" \
  || [ $? -lt 124 ] && bash tools/r04_prof.sh r04i
