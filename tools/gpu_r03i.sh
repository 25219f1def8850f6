set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u tools/c3_detail.py 64 200000 > $OUT/c3_detail_64.txt 2>&1
