# A/B of the shipped library against alternate builds (tools/libgll_alt*.so) at one config
#   bash tools/ab_session.sh <tag> <config> [batch]
cd "$GRAFT_REPO_ROOT"
T=$1; C=$2; B=${3:-1}
A="python3 tools/ab_flags.py --configs $C --batch $B --flags 0 --reps 10"
steps="$A"
for lib in tools/libgll_alt*.so; do [ -f "$lib" ] && steps="$steps && echo $lib && $A --lib $lib"; done
steps="$steps && echo main && $A"
bash tools/gpu_steps.sh "${T}:400:$steps"
