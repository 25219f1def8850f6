# Round 3: block-wide self test -- tile probe, GPU suite, C2 probe, C3 64.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u tools/tile_probe.py > $OUT/tile_probe.txt 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_4k.txt 2>&1
timeout -k 10 300 python -u bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --no-cpu --steps 1 --warmup 1 > $OUT/c3_q64.json 2> $OUT/c3_q64.err
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench_c2.json 2> $OUT/bench_c2.err
