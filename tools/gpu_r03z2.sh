set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u tools/tile_probe.py > $OUT/tile_probe.txt 2>&1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_4k.txt 2>&1
