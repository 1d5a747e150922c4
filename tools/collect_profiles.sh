# Copy one profile session's summaries (tools/prof_session.sh <tag>, merged back into
# gpurun_out/) into profiles/ under the names bench.py cites:
#   <tag>_<cfg>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
#   <tag>_pmc_<cfg>.json           FETCH_SIZE x 2 + WRITE_SIZE per launch (tools/pmc_summary.py)
#   <tag>_mfma_<cfg>.json          the Gram's MFMA counters (tools/mfma_summary.py)
#   bash tools/collect_profiles.sh <tag>
T=${1:?tag}
cd "$(dirname "$0")/.." || exit 1
for d in gpurun_out/${T}_prof_*; do
  [[ -d $d ]] || continue
  cfg=${d#gpurun_out/${T}_prof_}
  f=$(find "$d" -name '*kernel_stats.csv' | head -1)
  [[ -n $f ]] && cp "$f" "profiles/${T}_${cfg}_kernel_stats.csv" && echo "profiles/${T}_${cfg}_kernel_stats.csv"
done
for f in gpurun_out/${T}_pmc_*.json gpurun_out/${T}_mfma_*.json gpurun_out/${T}_build.json; do
  [[ -f $f ]] && cp "$f" profiles/ && echo "profiles/$(basename "$f")"
done
