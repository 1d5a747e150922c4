# Per-kernel timings at B = 1 and B = 64 (ns, fullysup, stress) and the select merge counters.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_flags.py --flags 0 --configs ns,fullysup,stress --batch 1,64 --reps 20 2>&1 | grep flags && \
timeout -k 10 120 python3 tools/merge_probe.py
