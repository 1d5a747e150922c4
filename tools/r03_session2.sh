# Round-3 session 2: pair test (now a flag), batched CG geometry A/B, row-panel probe.
bash tools/r03_run.sh \
 "t_pair:200:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k 'column_pair or batched_graphs'" \
 "bnt_ab:400:bash tools/r03_bnt_ab.sh" \
 "panel_probe:300:python -u tools/panel_probe.py"
