# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
# Every step has its own time limit; a fault, abort or time-out ends the session (no further GPU step).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
B="python -u bench.py --steps 1 --warmup 1 --no-cpu"
run c5 200 $B --workload c5 > $OUT/c5.json 2> $OUT/c5.err
run c3 200 $B --workload c3 > $OUT/c3.json 2> $OUT/c3.err
run c5s20 200 env SMP_SLICE_MS=20 $B --workload c5 > $OUT/c5s20.json 2> $OUT/c5s20.err
run c5s100 200 env SMP_SLICE_MS=100 $B --workload c5 > $OUT/c5s100.json 2> $OUT/c5s100.err
run c3s20 200 env SMP_SLICE_MS=20 $B --workload c3 > $OUT/c3s20.json 2> $OUT/c3s20.err
run c5np 200 env SMP_PRE_SCOUTS=0 $B --workload c5 > $OUT/c5np.json 2> $OUT/c5np.err
run c3np 200 env SMP_PRE_SCOUTS=0 $B --workload c3 > $OUT/c3np.json 2> $OUT/c3np.err
run t 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "full_budget or batch or reprovisioned or relaunch" > $OUT/t_batch.txt 2>&1
