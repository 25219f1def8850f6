# Device timeline of the pre-solution iterations 40-80 (SMP_TRACE build) of C2 seed 1.
set -e
OUT=gpurun_out
mkdir -p $OUT
SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_trace_pre.so timeout -k 10 120 python -u tools/trace_probe.py 100 > $OUT/trace_probe_pre.txt 2>&1
timeout -k 10 200 python -u tools/ttff_probe.py 4 > $OUT/ttff_probe.txt 2>&1 || true
