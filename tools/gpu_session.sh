# scratch driver of one gpurun call (edited per call): heartbeat + the steps below, each under its own time limit
OUT=$PWD/gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/r05_t_gpu_nnrec.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/r05_bench_nnrec.json 2> $OUT/r05_bench_nnrec.err &&
timeout -k 10 300 python -u bench.py > $OUT/r05_bench_nnrec2.json 2> $OUT/r05_bench_nnrec2.err &&
timeout -k 10 200 python -u tools/perf_probe.py 4000 > $OUT/r05_perf_nnrec.txt 2>&1
