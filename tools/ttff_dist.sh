# TTFF distribution on C2 for scout counts / pre-solution delays (tools/ttff_dist.py); outputs under gpurun_out/
set -e
for sd in "4 3" "2 2"; do set -- $sd; SMP_PRE_DELAY=$2 timeout -k 10 120 python tools/ttff_dist.py $1 8; done
