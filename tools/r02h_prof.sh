#!/bin/bash
# Round-2h profile session (GPU box): rocprofv3 kernel stats + FETCH/WRITE PMC for the NS bench
# command and the B = 64 NS batched probe, kernel stats for the FullySup single graph.  Each
# profiler pass has its own limit; any failure ends the script.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && R=$PWD
P="timeout -s KILL 150 rocprofv3"
NS="python3 $R/bench.py --config ns --steps 100 --warmup 10 --cpu-seconds 0 --no-profile --batch 0"
NSP="python3 $R/bench.py --config ns --steps 20 --warmup 5 --cpu-seconds 0 --no-profile --batch 0"
FS="python3 $R/bench.py --config fullysup --steps 100 --warmup 10 --cpu-seconds 0 --no-profile --batch 0"
B64="python3 $R/tools/batch_probe.py"
export PROBE_B=64 GLL_GRID_COOP=0
$P --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ns -o run -- $NS > gpurun_out/prof_ns.log 2>&1 && \
$P --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_ns -o run -- $NSP > gpurun_out/pmc_fetch_ns.log 2>&1 && \
$P --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_ns -o run -- $NSP > gpurun_out/pmc_write_ns.log 2>&1 && \
$P --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b64 -o run -- $B64 > gpurun_out/prof_b64.log 2>&1 && \
$P --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_b64 -o run -- $B64 > gpurun_out/pmc_fetch_b64.log 2>&1 && \
$P --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_b64 -o run -- $B64 > gpurun_out/pmc_write_b64.log 2>&1 && \
$P --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fullysup -o run -- $FS > gpurun_out/prof_fullysup.log 2>&1
rc=$?
echo "profile session rc=$rc"
python3 tools/pmc_summary.py gpurun_out/pmc_fetch_ns gpurun_out/pmc_write_ns gpurun_out/pmc_ns.json --config ns || rc=1
python3 tools/pmc_summary.py gpurun_out/pmc_fetch_b64 gpurun_out/pmc_write_b64 gpurun_out/pmc_ns_b64.json --config ns_b64 || rc=1
for d in prof_ns prof_b64 prof_fullysup; do f=$(find gpurun_out/$d -name '*kernel_stats.csv' | head -1); [[ -n $f ]] && cp "$f" gpurun_out/${d}_kernel_stats.csv && head -8 "$f" | cut -c1-160; done
exit $rc
