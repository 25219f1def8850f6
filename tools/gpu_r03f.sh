# Round 3: parallel scan collection -- parity of the split scans, then the 1e5 probe under participant counts.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "distributed or large_tree" > $OUT/dist_tests.log 2>&1
for v in "64 16" "64 8" "32 32" "16 16"; do
  set -- $v
  echo "== PNN $1 PNEAR $2" >> $OUT/scan_sweep.txt
  SMP_SCAN_PNN=$1 SMP_SCAN_PNEAR=$2 timeout -k 10 120 python -u tools/perf_probe.py 100000 >> $OUT/scan_sweep.txt 2>&1
done
echo "== no split" >> $OUT/scan_sweep.txt
SMP_SCAN_MIN=0 timeout -k 10 120 python -u tools/perf_probe.py 100000 >> $OUT/scan_sweep.txt 2>&1
