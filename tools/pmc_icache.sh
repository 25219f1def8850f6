set -e
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES -d $R/gpurun_out/pmc_ic -o ic -- python3 $R/tools/perf_probe.py 2000 > $R/gpurun_out/pmc_ic.log 2>&1
