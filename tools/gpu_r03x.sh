set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 python -u tools/startup_probe.py > $OUT/startup_probe.txt 2>&1
