# Scratch GPU session of the current experiment (rewritten per experiment; run from the repo root through gpurun).
OUT=gpurun_out
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/profile_round.sh r05 c2 && echo "profile rc=0" >> $OUT/status.txt
