# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "planner_parity or large_tree or relaunch" > $OUT/t_post.log 2>&1
for v in "SMP_POST=0" "SMP_POST=1" "SMP_POST_LEAD=8" "SMP_POST_LEAD=32" "SMP_POST_CAP=200" "SMP_POST_CAP=240"; do
  echo "== $v" >> $OUT/post_sweep.txt
  env $v timeout -k 10 120 python -u tools/perf_probe.py 4000 >> $OUT/post_sweep.txt 2>&1
done
SMP_SETS=expand-edges,connect-edges SMP_TILES=8,-1 timeout -k 10 200 python -u tools/tile_probe.py > $OUT/tile_probe.txt 2>&1
SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_rowb.so SMP_SETS=expand-edges SMP_TILES=8,-1 timeout -k 10 200 python -u tools/tile_probe.py > $OUT/tile_probe_rowb.txt 2>&1
SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_rowb.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "job_tile_shapes" > $OUT/t_rowb.log 2>&1
