set -e
OUT=gpurun_out
mkdir -p $OUT
SMP_HOST_PROF=1 timeout -k 10 120 python -u tools/host_overhead_probe.py > $OUT/host_overhead.txt 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
