# Round 3: C3 phase breakdown without helpers; C2 at 1e5 iterations with the scouts' phases.
set -e
OUT=gpurun_out
mkdir -p $OUT
SMP_HELPERS=-1 timeout -k 10 200 python -u tools/c3_detail.py 64 100000 > $OUT/c3_64_h-1.txt 2>&1
timeout -k 10 200 python -u tools/perf_probe.py 100000 > $OUT/perf_probe_1e5.txt 2>&1
