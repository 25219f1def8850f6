# Round 3: tile latency probe, helper pickup / tile-stage clocks (SMP_JOB_PROF build), C3 64 with the many-process CPU leg.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -u tools/tile_probe.py > $OUT/tile_probe.txt 2>&1
SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_jp.so SMP_JOB_PROF=1 timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_jp.txt 2>&1
timeout -k 10 400 python -u bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --steps 1 --warmup 1 > $OUT/c3_q64_cpu.json 2> $OUT/c3_q64_cpu.err
