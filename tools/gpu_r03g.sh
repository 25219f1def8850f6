# Round 3: split-scan tuning at 3e4 / 1e5 iterations, then the large-tree bench line (seed 7 = the 1e5 fixture).
set -e
OUT=gpurun_out
mkdir -p $OUT
for v in "64 8 12288" "64 4 12288" "48 8 12288" "64 8 6144" "64 8 24576"; do
  set -- $v
  echo "== PNN $1 PNEAR $2 MIN $3" >> $OUT/scan_sweep2.txt
  SMP_SCAN_PNN=$1 SMP_SCAN_PNEAR=$2 SMP_SCAN_MIN=$3 timeout -k 10 120 python -u tools/perf_probe.py 30000 100000 >> $OUT/scan_sweep2.txt 2>&1
done
timeout -k 10 400 python -u bench.py --iterations 100000 --seed 7 --steps 2 --warmup 1 > $OUT/bench_1e5.json 2> $OUT/bench_1e5.err
