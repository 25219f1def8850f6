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
step s4_micro 60 ./tools/micro/fp64_latency
SMP_LIB=$PWD/squirrel_motion_planner_amd/lib/libsmp_gpu_jps8.so SMP_JOB_PROF=1 step s7_jps8 200 python -u tools/perf_probe.py 4000
SMP_LIB=$PWD/squirrel_motion_planner_amd/lib/libsmp_gpu_jpp64.so SMP_JOB_PROF=1 step s8_jpp64 200 python -u tools/perf_probe.py 4000
SMP_LIB=$PWD/squirrel_motion_planner_amd/lib/libsmp_gpu_jp.so SMP_JOB_PROF=1 SMP_HELPERS=100 step s9_jph100 200 python -u tools/perf_probe.py 4000
