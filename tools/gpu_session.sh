# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
# Every step has its own time limit; a fault, abort or time-out ends the session (no further GPU step).
OUT=gpurun_out
mkdir -p $OUT
# heartbeat for long silent CPU legs (every step still has its own time limit)
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
run bench 500 python bench.py --steps 20 --warmup 2 > $OUT/bench_c2_20.json 2> $OUT/bench_c2_20.err
run c5 600 python bench.py --workload c5 --steps 1 --warmup 1 > $OUT/c5_q8.json 2> $OUT/c5_q8.err
run c3 400 python bench.py --workload c3 --steps 1 --warmup 1 > $OUT/c3_q8.json 2> $OUT/c3_q8.err
run ik 300 python tools/ik_report.py $OUT/ik_report.json > $OUT/ik.log 2>&1
for v in 6 20; do run ttff$v 200 env SMP_PRE_HELPERS=$v python -u tools/ttff_seeds.py 3 $OUT/ttff_pre$v.json > $OUT/ttff_pre$v.txt 2>&1; done
run trace 120 env SMP_TRACE_W0=16 SMP_TRACE_NW=4 SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_trace.so python -u tools/trace_probe.py > $OUT/trace_r04.txt 2>&1
