# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { local name=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac; }
run scans 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tree_scans.py > $OUT/r05_t_scans.txt 2>&1
run slp 120 python -u tools/slice_probe.py 512 4096 16384 > $OUT/r05_slice_probe4.txt 2>&1
run perf 300 python -u tools/perf_probe.py 4000 100000 200000 > $OUT/r05_perf_s3.txt 2>&1
run gpu 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/r05_t_gpu2.txt 2>&1
