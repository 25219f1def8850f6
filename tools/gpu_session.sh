# scratch driver of one gpurun call (edited per call): heartbeat + the steps below, each under its own time limit.
# A step's exit status 0 or 1 (a test failure) lets the next one run; anything else (a fault, an abort, a time limit)
# ends the call there.
OUT=$PWD/gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() {  # step NAME LIMIT CMD...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.txt 2>&1
  local rc=$?
  echo "step $name rc $rc" | tee -a $OUT/steps.txt
  [ $rc -le 1 ] || exit $rc
}
step t_sub 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tree_scans.py tests/test_gpu_parity.py -k "tree_scans or fp32 or distributed or large_tree or oracle_continues or planner_parity"
SMP_LIB=$PWD/squirrel_motion_planner_amd/lib/libsmp_gpu_trace1e5.so step s13_trace1e5 300 python -u tools/trace_probe.py 100100
step perf 200 python -u tools/perf_probe.py 4000 30000
step b3e5 200 python -u bench.py --iterations 300000 --steps 1 --warmup 0 --no-cpu
step nstep 200 python -u tools/near_step_probe.py 30000
