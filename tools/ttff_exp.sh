# TTFF distribution with per-scout debug output (experiments); outputs under gpurun_out/
set -e
SMP_DEBUG_SCOUTS=1 timeout -k 10 120 python tools/ttff_dist.py 4 12 > gpurun_out/ttff_dbg.log 2>&1
