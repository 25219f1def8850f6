# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
# Every step has its own time limit; a fault, abort or time-out ends the session (no further GPU step).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
B="python -u bench.py --steps 1 --warmup 1 --no-cpu --workload c5"
run d5 200 $B > $OUT/d5.json 2> $OUT/d5.err
run d3 200 env SMP_PRE_LEAD_DIV=3 $B > $OUT/d3.json 2> $OUT/d3.err
run d8 200 env SMP_PRE_LEAD_DIV=8 $B > $OUT/d8.json 2> $OUT/d8.err
run d12 200 env SMP_PRE_LEAD_DIV=12 $B > $OUT/d12.json 2> $OUT/d12.err
