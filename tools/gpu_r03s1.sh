# Session re-entry check: GPU suite, smoke, bench, iteration phase probe of the current build.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 60 ./tools/micro/call_overhead.bin > $OUT/call_overhead.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_4k.txt 2>&1
