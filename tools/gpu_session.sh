# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > $OUT/t_ea.log 2>&1
for v in "SMP_EARLY_ASK=0" "SMP_EARLY_ASK=1"; do
  echo "== $v" >> $OUT/ea_sweep.txt
  env $v timeout -k 10 120 python -u tools/perf_probe.py 4000 >> $OUT/ea_sweep.txt 2>&1
done
