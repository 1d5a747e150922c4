# round-4 GPU session j: whole-GPU CG iteration timeline at stress (trace build)
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh "r04j_gv_trace:120:python3 tools/gv_trace.py"
