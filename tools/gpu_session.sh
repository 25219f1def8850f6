# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
# Every step has its own time limit; a fault, abort or time-out ends the session (no further GPU step).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
run rc 200 env SMP_RING_CHECK=1 SMP_LIB=$PWD/squirrel_motion_planner_amd/lib/libsmp_gpu_rc.so python -u tools/divergence_probe.py 0 3000 2:0 > $OUT/div_rc.txt 2>&1
run dg 300 python -u tools/divergence_probe.py 0 20000 2:0 29:2 0:1 > $OUT/div_guard.txt 2>&1
run p0 100 env SMP_SCENE=c5 SMP_HELPERS=29 SMP_SCOUT=2 SMP_C5Q=0 python -u tools/perf_probe.py 20000 > $OUT/c5q0.txt 2>&1
