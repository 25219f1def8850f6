# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
# Every step has its own time limit; a fault, abort or time-out ends the session (no further GPU step).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
run c5 200 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu > $OUT/c5.json 2> $OUT/c5.err
run c5m0 200 env SMP_XCD_MARGIN=0 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu > $OUT/c5m0.json 2> $OUT/c5m0.err
run c5m2 200 env SMP_XCD_MARGIN=2 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu > $OUT/c5m2.json 2> $OUT/c5m2.err
run c3 200 python -u bench.py --workload c3 --steps 1 --warmup 1 --no-cpu > $OUT/c3.json 2> $OUT/c3.err
run c3m0 200 env SMP_XCD_MARGIN=0 python -u bench.py --workload c3 --steps 1 --warmup 1 --no-cpu > $OUT/c3m0.json 2> $OUT/c3m0.err
run c2 200 python -u bench.py --no-cpu > $OUT/c2.json 2> $OUT/c2.err
run t 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "full_budget or batch or reprovisioned" > $OUT/t_batch.txt 2>&1
