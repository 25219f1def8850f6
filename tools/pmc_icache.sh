# Instruction-cache and wait counters of the planner (C2, 2000 iterations, helpers off so that plan_kernel runs
# alone under counter collection), two passes; then the C2 bench of the library variants given as arguments.
set -e
export TMPDIR=/tmp
R=$PWD
mkdir -p $R/gpurun_out
cd /tmp
SMP_HELPERS=-1 timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES -d $R/gpurun_out/pmc_ic -o ic -- python3 $R/tools/perf_probe.py 2000 > $R/gpurun_out/pmc_ic.log 2>&1
SMP_HELPERS=-1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU -d $R/gpurun_out/pmc_wait -o wt -- python3 $R/tools/perf_probe.py 2000 > $R/gpurun_out/pmc_wait.log 2>&1
cd $R
bash tools/lib_sweep.sh "$@"
