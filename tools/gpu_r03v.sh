set -e
OUT=gpurun_out
mkdir -p $OUT
SMP_HOST_PROF=1 timeout -k 10 120 python -u tools/host_overhead_probe.py > $OUT/host_overhead.txt 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $OUT/bench_c2_10.json 2> $OUT/bench_c2_10.err
timeout -k 10 400 python -u bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --steps 1 --warmup 1 > $OUT/c3_q64.json 2> $OUT/c3_q64.err
