# scratch driver of one gpurun call (edited per call): heartbeat + the steps below, each under its own time limit
OUT=$PWD/gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 120 python -u tools/startup_probe.py > $OUT/r05_startup4.txt 2>&1 &&
timeout -k 10 200 python -u tools/perf_probe.py 100 > $OUT/r05_perf_s0.txt 2>&1 &&
timeout -k 10 300 python -u tools/ttff_seeds.py 1 $OUT/r05_ttff_s0.json > $OUT/r05_ttff_s0.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/r05_t_gpu_s0.txt 2>&1
