# Helper kernel with the scan-slice and sampler roles outlined (noinline) vs the current build: planner timing and
# SMP_JOB_PROF helper tile stages.
set -e
OUT=gpurun_out
mkdir -p $OUT
for v in jp jp_ni ni; do
  SMP_JOB_PROF=1 SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_$v.so timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_$v.txt 2>&1
done
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_base.txt 2>&1
