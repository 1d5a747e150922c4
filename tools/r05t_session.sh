# r05t: row-build checkpoints at stress (auto eps, as the bench) and FullySup, trace build
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TRACE_CFG=stress TRACE_EPS=0 timeout -k 10 120 python tools/trace_probe.py > gpurun_out/r05t_trace_stress.txt 2>&1 || exit $?
TRACE_CFG=fullysup timeout -k 10 120 python tools/trace_probe.py > gpurun_out/r05t_trace_fullysup.txt 2>&1 || exit $?
TRACE_CFG=ns timeout -k 10 120 python tools/trace_probe.py > gpurun_out/r05t_trace_ns.txt 2>&1 || exit $?
