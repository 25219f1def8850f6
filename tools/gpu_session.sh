# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 2 > $OUT/bench_c2_20.json 2> $OUT/bench_c2_20.err
timeout -k 10 300 python bench.py --workload c5 --steps 1 --warmup 1 > $OUT/c5_q8.json 2> $OUT/c5_q8.err
timeout -k 10 300 python bench.py --workload c3 --steps 1 --warmup 1 > $OUT/c3_q8.json 2> $OUT/c3_q8.err
timeout -k 10 300 python tools/ik_report.py $OUT/ik_report.json > $OUT/ik.log 2>&1
