set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u tools/ttff_probe.py 4 6 8 > $OUT/ttff_probe.txt 2>&1
