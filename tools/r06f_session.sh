# r06f: the bank-aware virtual-row order (vr_order_kernel) -- GPU tests of the balanced CG, A/B
# against the column order (GLL_FLAG_VR_ORDER_OFF = 524288) at FullySup B = 1 / 64, rocprof
# kernel stats of both, LDS bank-conflict counters of the FullySup bench with the order
cd "$GRAFT_REPO_ROOT"
R=$PWD
PM="--pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv"
bash tools/gpu_steps.sh \
  "r06f_tests:300:python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k 'balanced or bank_aware or batched_graphs_equal'" \
  "r06f_ab:300:python3 tools/ab_flags.py --flags 0,524288 --reps 20 --configs fullysup --batch 1,64" \
  "r06f_prof_on:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r06f_prof_on -o run -- python3 $R/bench.py --config fullysup --steps 60 --warmup 10 --cpu-seconds 0 --no-profile --batch 0" \
  "r06f_lds_on:150:rocprofv3 $PM -d gpurun_out/r06f_lds_fullysup -o run -- python3 $R/bench.py --config fullysup --steps 60 --warmup 10 --cpu-seconds 0 --no-profile --batch 0"
rc=$?
[ -d gpurun_out/r06f_lds_fullysup ] && python3 tools/counter_summary.py gpurun_out/r06f_lds_fullysup > gpurun_out/r06f_lds_fullysup.txt
exit $rc
