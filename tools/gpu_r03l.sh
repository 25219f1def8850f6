# Round 3: link-pair prefilter of the self test -- tile probe, check/planner parity, C2 probe, C3 detail.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u tools/tile_probe.py > $OUT/tile_probe.txt 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_4k.txt 2>&1
timeout -k 10 200 python -u tools/c3_detail.py 64 200000 > $OUT/c3_detail_64.txt 2>&1
