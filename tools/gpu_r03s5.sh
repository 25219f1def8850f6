# Single-launch single queries: relaunch-equivalence test, GPU suite, timing.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k relaunched -x -v --timeout 120 --timeout-method thread > $OUT/relaunch_test.log 2>&1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_4k.txt 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench10.json 2> $OUT/bench.err
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
