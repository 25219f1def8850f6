# scratch driver of one gpurun call (edited per call): heartbeat + the steps below, each under its own time limit
OUT=$PWD/gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PMC_LIMIT=300 BENCH_LIMIT=500 KT_LIMIT=200 bash tools/profile_round.sh r05 c2_iter300000 --iterations 300000 --steps 1 --warmup 0 && echo "3e5 rc=0" >> $OUT/status.txt &&
SKIP_PMC=1 SKIP_BENCH=1 KT_LIMIT=400 bash tools/profile_round.sh r05 c2_iter1000000 --iterations 1000000 --steps 1 --warmup 0 && echo "1e6kt rc=0" >> $OUT/status.txt
