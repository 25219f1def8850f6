# One GPU call: parity tests, the headline bench and the C4 convergence report (run from the repo root through gpurun).
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 200 python tools/configs_report.py c4 $OUT/c4_convergence.json --seconds 2 > $OUT/c4.log 2>&1
