# IK build of HEAD (goal terms in registers, joint update inside the FK step): full GPU suite, smoke, IK report.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/s20_gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/s20_smoke.log 2>&1
timeout -k 10 400 python tools/ik_report.py $OUT/r03c_ik_report.json > $OUT/r03c_ik_report.log 2>&1
SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_ikx3prof.so timeout -k 10 120 python tools/ik_phase_probe.py > $OUT/r03c_ik_phase.txt 2>&1
