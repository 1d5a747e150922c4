# round-4 GPU session s: the Gram tail's subtiles over k-slices; order_perm batched -- tests,
# stress A/B; select D2 row loads nontemporal (alt build) -- time and counter bytes
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "r04s_tests:400:python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k 'tail or gram or locality or stress or fixture'" \
  "r04s_ab_tail:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --knob 4 --values 0,2,1,0,2 --reps 10" \
  "r04s_ab_nt:300:python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --reps 10 && python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --reps 10 --lib tools/libgll_alt.so && python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --reps 10" \
  "r04s_pmcf_main:120:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r04s_pmcf_main -o run -- python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --reps 3" \
  "r04s_pmcf_alt:120:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r04s_pmcf_alt -o run -- python3 tools/ab_flags.py --configs stress --batch 1 --flags 0 --reps 3 --lib tools/libgll_alt.so"
