# Map sweeps with the candidates' brick words staged in one round trip: parity suite, tile and planner timing.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests_staged.log 2>&1
timeout -k 10 200 python -u tools/tile_probe.py > $OUT/tile_probe_c2_staged.txt 2>&1
SMP_SCENE=c5 timeout -k 10 300 python -u tools/tile_probe.py > $OUT/tile_probe_c5_staged.txt 2>&1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_staged.txt 2>&1
