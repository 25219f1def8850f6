set -e
OUT=gpurun_out
mkdir -p $OUT
SMP_HELPERS_FIRST=1 timeout -k 10 120 python -u tools/startup_probe.py > $OUT/startup_probe_hf.txt 2>&1
SMP_HELPERS_FIRST=1 timeout -k 10 200 python -u tools/ttff_probe.py 4 > $OUT/ttff_probe_hf.txt 2>&1
SMP_HELPERS_FIRST=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $OUT/bench_c2_hf.json 2> $OUT/bench_c2_hf.err
