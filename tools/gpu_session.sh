# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
set -e
OUT=gpurun_out
mkdir -p $OUT
export SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_jp.so SMP_JOB_PROF=1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/jp_adaptive.txt 2>&1
SMP_TILE_CT=8 timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/jp_ct8.txt 2>&1
