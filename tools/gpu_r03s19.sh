# IK experiment 4: as r03s18 plus the FK chain loading local frames two steps ahead, rotation step selected not
# branched; phase clocks of HEAD / variant 3 / variant 4 and goal-search reports of HEAD / variant 4 on one box.
set -e
OUT=gpurun_out
mkdir -p $OUT
V=squirrel_motion_planner_amd/lib
SMP_LIB=$V/libsmp_gpu_ikx4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ik.py -x -q --timeout 200 --timeout-method thread > $OUT/ikx4_tests.log 2>&1
for v in ikprof ikx3prof ikx4prof; do
  SMP_LIB=$V/libsmp_gpu_$v.so timeout -k 10 120 python tools/ik_phase_probe.py > $OUT/ik_phase_s19_$v.txt 2>&1
done
SMP_LIB=$V/libsmp_gpu_ikx4.so timeout -k 10 400 python tools/ik_report.py $OUT/ik_report_ikx4.json > $OUT/ik_report_ikx4.log 2>&1
timeout -k 10 400 python tools/ik_report.py $OUT/ik_report_head.json > $OUT/ik_report_head.log 2>&1
