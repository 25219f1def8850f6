# Round-end rehearsal of HEAD: GPU suite, smoke, default bench line.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/final_gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/final_smoke.log 2>&1
timeout -k 10 300 python bench.py > $OUT/final_bench.json 2> $OUT/final_bench.err
