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
KT_LIMIT=600 BENCH_LIMIT=900 PMC_LIMIT=600 step prof_1e6 1150 bash tools/profile_round.sh r06 c2_iter1000000 --iterations 1000000 --steps 1 --warmup 0
