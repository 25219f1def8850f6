# GPU tests + bench for the current build (experiments); outputs under gpurun_out/
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_exp.log 2>&1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_exp.log 2>&1
