# Round 3: run-ahead sampler threshold on C3 (64 queries, 3 helpers each) and C2.
set -e
OUT=gpurun_out
mkdir -p $OUT
for m in 2 4 8; do
  SMP_SAMPLER_MIN=$m timeout -k 10 300 python -u bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --no-cpu --steps 1 --warmup 1 > $OUT/c3_q64_s$m.json 2> $OUT/c3_q64_s$m.err
done
SMP_SAMPLER_MIN=4 timeout -k 10 200 python -u tools/c3_detail.py 64 200000 > $OUT/c3_detail_64_s4.txt 2>&1
