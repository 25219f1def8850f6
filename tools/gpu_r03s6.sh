# Path gathered on the device: parity subset, host stage stamps of a C2 call, bench.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shim_cpp.py tests/test_gpu_multi.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/parity_subset.log 2>&1
SMP_HOST_PROF=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu > $OUT/bench_hostprof.json 2> $OUT/bench_hostprof.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench10.json 2> $OUT/bench.err
