# Round 3 profiles: small-tree phase probe, then the round's bench line, kernel-trace stats and HBM counter passes.
set -e
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_4k.txt 2>&1
bash tools/profile_round.sh r03
