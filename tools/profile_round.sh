# Round profiles on the GPU box (run from the repo root through gpurun):
#   bench line, rocprofv3 kernel-trace stats of the bench, and the two HBM counter passes of plan_kernel
#   (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950; counter collection serialises dispatches, so those
#   passes run with --helpers -1: all tile work inside plan_kernel).  Outputs under gpurun_out/ (merged back by
#   gpurun); then, locally: tools/rocpd_summary.py stats / pmc on the merged .db files -> profiles/ROUND_*.
set -e
ROUND=${1:-r01}
R=$PWD
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_kt -o kt -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_pmc -o pmc -- python3 $R/bench.py --no-cpu --helpers -1 --steps 1 --warmup 0 > $OUT/pmc.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_pmcw -o pmcw -- python3 $R/bench.py --no-cpu --helpers -1 --steps 1 --warmup 0 > $OUT/pmcw.log 2>&1
cd $R
