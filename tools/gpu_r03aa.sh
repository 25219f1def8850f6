set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 250 --timeout-method thread -k "reprovisioned or c3_random or batch_equals" > $OUT/reprov_tests.log 2>&1
