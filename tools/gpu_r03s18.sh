# IK experiment 3: as r03s17 plus the goal terms of the error read once per run (were global loads per iteration).
set -e
OUT=gpurun_out
mkdir -p $OUT
V=squirrel_motion_planner_amd/lib
SMP_LIB=$V/libsmp_gpu_ikx3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ik.py -x -q --timeout 200 --timeout-method thread > $OUT/ikx3_tests.log 2>&1

SMP_LIB=$V/libsmp_gpu_ikx3prof.so timeout -k 10 120 python tools/ik_phase_probe.py > $OUT/ik_phase_ikx3.txt 2>&1
SMP_LIB=$V/libsmp_gpu_ikx3.so timeout -k 10 400 python tools/ik_report.py $OUT/ik_report_ikx3.json > $OUT/ik_report_ikx3.log 2>&1
