# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/profile_round.sh r04 c2 && echo c2 done >> $OUT/status.txt && \
bash tools/profile_round.sh r04 c3 --workload c3 && echo c3 done >> $OUT/status.txt && \
bash tools/profile_round.sh r04 c5 --workload c5 && echo c5 done >> $OUT/status.txt
