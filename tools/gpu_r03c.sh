# Round 3: C3 (64 queries on one GPU) helper sweep.
set -e
OUT=gpurun_out
mkdir -p $OUT
for h in -1 1 3 0; do
  timeout -k 10 200 python bench.py --workload c3 --queries-per-gpu 64 --helpers $h --steps 1 --warmup 1 --no-cpu --samples 200000 > $OUT/c3_h$h.json 2>> $OUT/c3.err
done
for s in 0; do
  timeout -k 10 200 python bench.py --workload c3 --queries-per-gpu 64 --helpers 3 --scout 0 --steps 1 --warmup 1 --no-cpu --samples 200000 > $OUT/c3_h3_s0.json 2>> $OUT/c3.err
done
