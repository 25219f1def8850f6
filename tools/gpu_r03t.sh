set -e
OUT=gpurun_out
mkdir -p $OUT
SMP_HOST_PROF=1 timeout -k 10 120 python -u tools/host_overhead_probe.py > $OUT/host_overhead.txt 2>&1
