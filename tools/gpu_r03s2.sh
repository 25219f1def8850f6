# Device timeline of the current build (SMP_TRACE) and the C2 tile stage probe.
set -e
OUT=gpurun_out
mkdir -p $OUT
SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_trace.so timeout -k 10 120 python -u tools/trace_probe.py > $OUT/trace_probe.txt 2>&1
timeout -k 10 200 python -u tools/tile_probe.py > $OUT/tile_probe_c2.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_shim_cpp.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/shim_multi.log 2>&1
