# threshold-scan select at 6 waves per SIMD (default) and 8 (tools/libgll_w8.so, 64 VGPRs)
set -o pipefail
run() { timeout -k 10 300 "$@" 2>&1 | grep -v amdgpu.ids; }
C=ns:64,fullysup:64
echo "== w6"; run python -u tools/select_ab.py --tag w6 --cases $C || exit $?
echo "== w8"; GLL_LIB_PATH=tools/libgll_w8.so run python -u tools/select_ab.py --tag w8 --against w6 --cases $C || exit $?
for dg in 1 2; do
echo "== w6 diag $dg"; GLL_SEL_DIAG=$dg run python -u tools/select_ab.py --tag d --cases $C || exit $?
echo "== w8 diag $dg"; GLL_LIB_PATH=tools/libgll_w8.so GLL_SEL_DIAG=$dg run python -u tools/select_ab.py --tag d --cases $C || exit $?
done
