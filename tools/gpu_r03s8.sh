# Session-2 round profiles of the current build: GPU suite, then tools/profile_round.sh (bench line, kernel-trace
# stats, FETCH_SIZE / WRITE_SIZE passes).
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
bash tools/profile_round.sh r03b
