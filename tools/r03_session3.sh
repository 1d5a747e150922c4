# Round-3 session 3: all GPU tests on the new dispatch + Gram epilogue, Gram epilogue A/B, CG geometry by B.
bash tools/r03_run.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "gramdiag:400:bash tools/r03_gramdiag_ab.sh" \
 "geo:200:python -u tools/ab_flags.py --flags 0 --configs ns --batch 1,8,16,25,32,64 --reps 20"
