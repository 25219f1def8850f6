# Refresh of the other BASELINE configurations with the current build (round 3, session 2).
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --steps 1 --warmup 1 > $OUT/c3_q64.json 2> $OUT/c3_q64.err
timeout -k 10 300 python bench.py --workload c3 --steps 1 --warmup 1 > $OUT/c3_q8.json 2> $OUT/c3_q8.err
timeout -k 10 400 python bench.py --workload c5 --steps 1 --warmup 1 > $OUT/c5_q8.json 2> $OUT/c5_q8.err
timeout -k 10 200 python tools/configs_report.py c4 $OUT/c4_convergence.json --seconds 2 > $OUT/c4.log 2>&1
timeout -k 10 300 python bench.py --iterations 100000 --seed 7 --steps 1 --warmup 1 > $OUT/c2_iter1e5.json 2> $OUT/c2_iter1e5.err
