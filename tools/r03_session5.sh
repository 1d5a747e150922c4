# Round-3 session 5: fp16 D2 storage tests, then its A/B, then every GPU test.
bash tools/r03_run.sh \
 "t_d2h:300:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k 'fp16 or batched or presplit or gram_256'" \
 "d2h_ab:500:bash tools/r03_d2h_ab.sh" \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread"
