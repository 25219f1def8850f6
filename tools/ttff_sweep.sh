set -e
mkdir -p gpurun_out
for d in 0 1 2 3; do echo "pre_delay $d"; SMP_PRE_DELAY=$d timeout -k 10 100 python tools/ttff_probe.py 2 3 4 6; done > gpurun_out/ttff_sweep.log 2>&1
