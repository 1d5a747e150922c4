# host-side cost of a step, with the backward as two launches and as the fused one
echo "== default (fused backward)"; python -u tools/host_breakdown.py 2>&1 | grep -v amdgpu.ids || exit $?
echo "== GLL_BWD_FUSED=0 (two launches)"; GLL_BWD_FUSED=0 python -u tools/host_breakdown.py 2>&1 | grep -v amdgpu.ids || exit $?
echo "== mt probe"; python -u tools/mt_probe.py 2>&1 | grep -v amdgpu.ids
