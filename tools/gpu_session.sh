# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "job_tile_shapes or check_configs_parity or disabled" > $OUT/t_tiles.log 2>&1
SMP_TILES=8,-8,-1 timeout -k 10 200 python -u tools/tile_probe.py > $OUT/tile_probe.txt 2>&1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_4k.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
