# IK: the joint update's six divisions issued together (one uniform branch, was one branch per term): IK tests,
# phase clocks of round-2 HEAD and this build, goal-search report.
set -e
OUT=gpurun_out
mkdir -p $OUT
V=squirrel_motion_planner_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_ik.py tests/test_shim_cpp.py -x -q --timeout 200 --timeout-method thread > $OUT/s21_tests.log 2>&1
for v in ikprof ikx5prof; do
  SMP_LIB=$V/libsmp_gpu_$v.so timeout -k 10 120 python tools/ik_phase_probe.py > $OUT/ik_phase_s21_$v.txt 2>&1
done
timeout -k 10 400 python tools/ik_report.py $OUT/r03c_ik_report.json > $OUT/r03c_ik_report.log 2>&1
