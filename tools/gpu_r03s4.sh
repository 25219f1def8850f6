# Parity + timing of the current build (edge_costs per wavefront).
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_4k.txt 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench10.json 2> $OUT/bench.err
for s in 6 16; do
  SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_s$s.so timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_4k_s$s.txt 2>&1
done
