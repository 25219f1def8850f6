# IK experiment 2: as r03s16 plus the joint update merged into the FK local-frame step.
set -e
OUT=gpurun_out
mkdir -p $OUT
V=squirrel_motion_planner_amd/lib
SMP_LIB=$V/libsmp_gpu_ikx2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ik.py -x -q --timeout 200 --timeout-method thread > $OUT/ikx2_tests.log 2>&1

SMP_LIB=$V/libsmp_gpu_ikx2prof.so timeout -k 10 120 python tools/ik_phase_probe.py > $OUT/ik_phase_ikx2.txt 2>&1
SMP_LIB=$V/libsmp_gpu_ikx2.so timeout -k 10 400 python tools/ik_report.py $OUT/ik_report_ikx2.json > $OUT/ik_report_ikx2.log 2>&1
