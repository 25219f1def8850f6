# Longer device timeline (6 iterations) of the post-solution cycle: when scouts get requests, finish, idle.
set -e
OUT=gpurun_out
mkdir -p $OUT
SMP_TRACE_W0=16 SMP_TRACE_NW=6 SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_trace.so timeout -k 10 120 python -u tools/trace_probe.py > $OUT/trace_probe_6it.txt 2>&1
