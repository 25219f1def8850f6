# Stop-first-valid jobs decided early (choose-parent / connect near loop, scout choose jobs): parity suite + timing.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_sfv.log 2>&1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_sfv.txt 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_sfv.json 2> $OUT/bench_sfv.err
timeout -k 10 400 python bench.py --workload c5 --steps 1 --warmup 1 --no-cpu > $OUT/c5_q8_sfv.json 2> $OUT/c5_q8_sfv.err
