# r05w: hub-row overflow scan / label loads batched (row_build); tools/libgll_alt_head.so = before
cd "$GRAFT_REPO_ROOT"
A="python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --reps 5"
bash tools/gpu_steps.sh \
  "r05w_tests:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k 'hub or stress or fixture or duplicate or batched_two_row'" \
  "r05w_trace_stress:120:TRACE_CFG=stress TRACE_EPS=0 python tools/trace_probe.py" \
  "r05w_ab_new:200:$A" "r05w_ab_head:200:$A --lib tools/libgll_alt_head.so" "r05w_ab_new2:200:$A"
