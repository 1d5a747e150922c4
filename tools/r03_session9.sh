# Round-3 final check on the clean build: smoke, every GPU test (incl. the batched independence test), bench.
STEPS=smoke,tests,bench bash tools/gpu_check.sh
