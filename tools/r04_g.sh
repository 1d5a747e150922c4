# round-4 GPU session g: kernel time through the apply vs the C ABI (path_probe)
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r04g_path_b64:200:PROBE_B=64 python3 tools/path_probe.py" \
  "r04g_path_b1:200:PROBE_B=1 python3 tools/path_probe.py"
