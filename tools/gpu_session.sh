# scratch driver of one gpurun call (edited per call): heartbeat + the steps below, each under its own time limit
OUT=$PWD/gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/r05_t_gpu_m32.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/perf_probe.py 4000 100000 > $OUT/r05_perf_m32.txt 2>&1 || exit 1
timeout -k 10 200 env SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_trace15.so SMP_TRACE_W0=20 python -u tools/trace_probe.py 100000 > $OUT/r05_trace_1e5e.txt 2>&1
