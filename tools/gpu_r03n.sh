# Round 3: many-query groups -- C3 64 queries by group size, then the GPU suite.
set -e
OUT=gpurun_out
mkdir -p $OUT
for m in 64 16 8 4; do
  SMP_MAX_ACTIVE=$m timeout -k 10 300 python -u bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --no-cpu --steps 1 --warmup 1 > $OUT/c3_q64_m$m.json 2> $OUT/c3_q64_m$m.err
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
