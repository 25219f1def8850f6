# C5 map-stage evidence (SURVEY 8d C5 / VERDICT r02 item 8): tile stage clocks on the 2 cm scene, the batch checker's
# rate on C5 configurations, then its counter passes (each pass its own run; outputs under gpurun_out/c5pmc).
set -e
R=$PWD
OUT=$R/gpurun_out
mkdir -p $OUT/c5pmc
SMP_SCENE=c5 timeout -k 10 200 python -u tools/tile_probe.py > $OUT/c5_tile_probe.txt 2>&1
timeout -k 10 200 python -u tools/c5_check_probe.py > $OUT/c5_check_probe.txt 2>&1
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/c5pmc/fetch -o p -- python3 $R/tools/c5_check_probe.py > $OUT/c5pmc/fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/c5pmc/tcc -o p -- python3 $R/tools/c5_check_probe.py > $OUT/c5pmc/tcc.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $OUT/c5pmc/tcp -o p -- python3 $R/tools/c5_check_probe.py > $OUT/c5pmc/tcp.log 2>&1
cd $R
