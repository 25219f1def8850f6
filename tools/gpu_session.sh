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
run gpu 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
run c5tw 200 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu > $OUT/c5_twin.json 2> $OUT/c5_twin.err
run c5one 200 env SMP_TWIN=0 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu > $OUT/c5_one.json 2> $OUT/c5_one.err
run c3tw 200 python -u bench.py --workload c3 --steps 1 --warmup 1 --no-cpu > $OUT/c3_twin.json 2> $OUT/c3_twin.err
run c3one 200 env SMP_TWIN=0 python -u bench.py --workload c3 --steps 1 --warmup 1 --no-cpu > $OUT/c3_one.json 2> $OUT/c3_one.err
