# IK experiment: Jacobian and error in one instruction stream (branch-free quaternion) vs HEAD.
set -e
OUT=gpurun_out
mkdir -p $OUT
V=squirrel_motion_planner_amd/lib
SMP_LIB=$V/libsmp_gpu_ikx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ik.py -x -q --timeout 200 --timeout-method thread > $OUT/ikx_tests.log 2>&1
SMP_LIB=$V/libsmp_gpu_ikprof.so timeout -k 10 120 python tools/ik_phase_probe.py > $OUT/ik_phase_base.txt 2>&1
SMP_LIB=$V/libsmp_gpu_ikxprof.so timeout -k 10 120 python tools/ik_phase_probe.py > $OUT/ik_phase_ikx.txt 2>&1
SMP_LIB=$V/libsmp_gpu_ikx.so timeout -k 10 400 python tools/ik_report.py $OUT/ik_report_ikx.json > $OUT/ik_report_ikx.log 2>&1
