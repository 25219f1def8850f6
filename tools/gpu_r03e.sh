# Round 3: distributed scans -- new parity tests first, then the whole GPU suite, then the 1e5-iteration probe.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "distributed or large_tree" > $OUT/dist_tests.log 2>&1
timeout -k 10 200 python -u tools/perf_probe.py 100000 > $OUT/perf_probe_1e5.txt 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
