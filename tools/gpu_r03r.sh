# Round 3: re-provisioning quota sweep on C3 (64 queries) and C5 (8 queries).
set -e
OUT=gpurun_out
mkdir -p $OUT
for d in 2 4 8 64; do
  SMP_REBALANCE_DIV=$d timeout -k 10 300 python -u bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --no-cpu --steps 1 --warmup 1 > $OUT/c3_q64_d$d.json 2> $OUT/c3_q64_d$d.err
  SMP_REBALANCE_DIV=$d timeout -k 10 300 python -u bench.py --workload c5 --no-cpu --steps 1 --warmup 1 > $OUT/c5_q8_d$d.json 2> $OUT/c5_q8_d$d.err
done
