# scratch driver of one gpurun call (edited per call): heartbeat + the steps below, each under its own time limit
OUT=$PWD/gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u bench.py --workload c3 > $OUT/r05_bench_c3_final2.json 2> $OUT/r05_bench_c3_final2.err &&
timeout -k 10 400 python -u bench.py --workload c5 > $OUT/r05_bench_c5_final2.json 2> $OUT/r05_bench_c5_final2.err &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r05_smoke_final3.txt 2>&1
