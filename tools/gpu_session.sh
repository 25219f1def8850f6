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
step s1_tests 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_tree_scans.py tests/test_gpu_collisions.py tests/test_gpu_parity.py -k "tree_scans or fp32 or collision or tile or check or distributed_scans or planner_parity or bench_workload"
step s2_perf 200 python -u tools/perf_probe.py 4000 30000
step s6_tile 300 python -u tools/tile_probe.py
step b1_3e5 200 python -u bench.py --iterations 300000 --steps 1 --warmup 0 --no-cpu
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/s15_counters.txt 2>&1; echo "list rc $?" >> $OUT/steps.txt
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/s16_pmc -o pmc -- python3 $GRAFT_REPO_ROOT/tools/perf_probe.py 4000 > $OUT/s16_pmc.log 2>&1; echo "pmc rc $?" >> $OUT/steps.txt
