# Round 3: re-provisioning of running queries -- C3 64 with / without, C5 8, then the GPU suite.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --no-cpu --steps 1 --warmup 1 > $OUT/c3_q64_rb.json 2> $OUT/c3_q64_rb.err
SMP_REBALANCE=0 timeout -k 10 300 python -u bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --no-cpu --steps 1 --warmup 1 > $OUT/c3_q64_norb.json 2> $OUT/c3_q64_norb.err
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 1 --warmup 1 > $OUT/c3_q8_rb.json 2> $OUT/c3_q8_rb.err
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
