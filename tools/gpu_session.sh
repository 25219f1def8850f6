# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
for ld in 3 5 8; do
  run perf_ld$ld 120 env SMP_LEAD_DIV=$ld python -u tools/perf_probe.py 4000 > $OUT/r05_perf4k_ld$ld.txt 2>&1
done
run perf_cc 120 env SMP_CONN_CHECK=1 SMP_LEAD_DIV=8 python -u tools/perf_probe.py 4000 > $OUT/r05_perf4k_cc_ld8.txt 2>&1
for pd in 2 4 5; do
  run ttff_pd$pd 200 env SMP_PRE_DELAY=$pd python -u tools/ttff_seeds.py 1 $OUT/r05_ttff_pd$pd.json > $OUT/r05_ttff_pd$pd.txt 2>&1
done
run ttff_pld 200 env SMP_PRE_LEAD_DIV=10 python -u tools/ttff_seeds.py 1 $OUT/r05_ttff_pld10.json > $OUT/r05_ttff_pld10.txt 2>&1
run perf 300 python -u tools/perf_probe.py 100000 200000 > $OUT/r05_perf_s4.txt 2>&1
