# scratch driver of one gpurun call (edited per call): heartbeat + the steps below, each under its own time limit
OUT=$PWD/gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PMC_LIMIT=200 BENCH_LIMIT=300 KT_LIMIT=200 bash tools/profile_round.sh r05 c2 && echo "c2 rc=0" >> $OUT/status.txt &&
PMC_LIMIT=200 BENCH_LIMIT=300 KT_LIMIT=200 bash tools/profile_round.sh r05 c3 --workload c3 --queries-per-gpu 8 && echo "c3 rc=0" >> $OUT/status.txt &&
PMC_LIMIT=200 BENCH_LIMIT=300 KT_LIMIT=200 bash tools/profile_round.sh r05 c5 --workload c5 --queries-per-gpu 8 && echo "c5 rc=0" >> $OUT/status.txt
