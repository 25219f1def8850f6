# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
# Every step has its own time limit; a fault, abort or time-out ends the session (no further GPU step).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
run twin 700 env SMP_TWIN=1 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/twin_tests.txt 2>&1
run slice0 700 env SMP_SLICE_MS=0 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "batch or queries or reprovisioned or full_budget" > $OUT/slice0_tests.txt 2>&1
