# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
run smoke 120 python -u __graft_entry__.py smoke > $OUT/r05_smoke.txt 2>&1
run gpu 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/r05_t_gpu3.txt 2>&1
for ld in 3 8; do
  run perf_ld$ld 120 env SMP_LEAD_DIV=$ld python -u tools/perf_probe.py 4000 > $OUT/r05_perf4k_ld$ld.txt 2>&1
done
for pd in 3 4 5; do
  run ttff_pd$pd 200 env SMP_PRE_DELAY=$pd python -u tools/ttff_seeds.py 1 $OUT/r05_ttff_pd$pd.json > $OUT/r05_ttff_pd$pd.txt 2>&1
done
run perf 300 python -u tools/perf_probe.py 100000 200000 > $OUT/r05_perf_s4.txt 2>&1
