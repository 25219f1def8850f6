# Round 3 probes: the planner at growing iteration budgets (tree sizes) and C3 with 64 queries on one GPU.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u tools/perf_probe.py 2000 10000 30000 100000 > $OUT/perf_probe.txt 2>&1
timeout -k 10 200 python -u tools/c3_detail.py 64 200000 > $OUT/c3_64.txt 2>&1
