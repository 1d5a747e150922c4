# r06zf (part 1): validation of the build with the DPP reduction read -- the whole GPU suite, smoke,
# utils.laplace at the reference's evaluation size, profile session for ns, ns_b64, fullysup
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_steps.sh \
  "r06zf_gpu_tests:420:python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "r06zf_smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "r06zf_laplace:300:python3 -u tools/laplace_probe.py"
rc=$?
[ $rc -ge 124 ] && exit $rc
bash tools/prof_session.sh r06zf ns ns_b64 fullysup
