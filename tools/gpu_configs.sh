# BASELINE configs beyond the headline bench (run from the repo root through gpurun); outputs under gpurun_out/.
#   C3 share of one GPU (8 random queries) and all 64 C3 queries on one GPU, C4 convergence, C5 tile-size sweep.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python bench.py --workload c3 --no-cpu --steps 1 --warmup 1 > $OUT/c3_q8.json 2> $OUT/c3_q8.err
timeout -k 10 400 python bench.py --workload c3 --queries-per-gpu 64 --samples 200000 --steps 1 --warmup 1 > $OUT/c3_q64.json 2> $OUT/c3_q64.err
timeout -k 10 200 python tools/configs_report.py c4 $OUT/c4_convergence.json --seconds 2 > $OUT/c4.log 2>&1
timeout -k 10 600 python tools/configs_report.py c5-sweep $OUT/c5_sweep.json --iterations 3000 \
  --libs squirrel_motion_planner_amd/lib/libsmp_gpu.so,squirrel_motion_planner_amd/lib/libsmp_gpu_ct16.so > $OUT/c5.log 2>&1
