# round-4 GPU session h: rocprofv3 kernel durations beside the dispatch-packet events, same run
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "r04h_path_b64_rocprof:240:PROBE_B=64 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04h_rp_b64 -o run -- python3 tools/path_probe.py" \
  "r04h_path_b1_rocprof:240:PROBE_B=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04h_rp_b1 -o run -- python3 tools/path_probe.py"
