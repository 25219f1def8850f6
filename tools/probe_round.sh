# Planner phase probe (C2, 4203 iterations) of the default build and of the SMP_JOB_PROF build, outputs under gpurun_out/
set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/perf_probe.py 4203 > gpurun_out/perf_default.log 2>&1
SMP_JOB_PROF=1 SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_jp.so timeout -k 10 200 python tools/perf_probe.py 4203 > gpurun_out/perf_jp.log 2>&1
