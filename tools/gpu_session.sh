# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
# Every step has its own time limit; a fault, abort or time-out ends the session (no further GPU step).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
run q4 200 env SMP_QSEL=1,2,4,7 SMP_SCOUT=4 python -u tools/batch_probe.py > $OUT/q4s4.txt 2>&1
run q6 200 env SMP_QSEL=1,2,4,7 SMP_SCOUT=6 python -u tools/batch_probe.py > $OUT/q4s6.txt 2>&1
run q8 200 env SMP_QSEL=1,2,4,7 SMP_SCOUT=8 python -u tools/batch_probe.py > $OUT/q4s8.txt 2>&1
