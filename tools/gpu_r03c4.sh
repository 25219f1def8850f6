set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python tools/configs_report.py c4 $OUT/c4_convergence.json --seconds 2 > $OUT/c4.log 2>&1
