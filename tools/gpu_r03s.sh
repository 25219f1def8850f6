set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $OUT/bench_c2_10.json 2> $OUT/bench_c2_10.err
