# tree-scan parity + timing (tools/near_probe.py) of the default library and of any variants named as arguments
set -e
T=gpurun_out/tree.npz
timeout -k 10 300 python -m pytest tests/test_gpu_tree_scans.py -x -q > gpurun_out/scan_tests.log 2>&1
timeout -k 10 120 python tools/near_probe.py 10000 $T > gpurun_out/np_base.log 2>&1
for v in "$@"; do SMP_LIB=$PWD/squirrel_motion_planner_amd/lib/libsmp_gpu_$v.so timeout -k 10 120 python tools/near_probe.py 10000 $T > gpurun_out/np_$v.log 2>&1; done
