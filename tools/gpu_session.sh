# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
# Every step has its own time limit; a fault, abort or time-out ends the session (no further GPU step).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
B="python -u bench.py --steps 2 --warmup 1 --no-cpu --workload c3"
run s50 200 $B > $OUT/s50.json 2> $OUT/s50.err
run s100 200 env SMP_SLICE_MS=100 $B > $OUT/s100.json 2> $OUT/s100.err
run s200 200 env SMP_SLICE_MS=200 $B > $OUT/s200.json 2> $OUT/s200.err
run s0 200 env SMP_SLICE_MS=0 $B > $OUT/s0.json 2> $OUT/s0.err
