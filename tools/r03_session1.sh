# Round-3 session: new batched-CG / panel tests first, then the CG A/B, then smoke + full GPU tests + bench.
bash tools/r03_run.sh \
 "t_new:400:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k 'column_pair or panel or batched'" \
 "nc_ab:400:bash tools/r03_nc_ab.sh" \
 && STEPS=smoke,tests,bench bash tools/gpu_check.sh
