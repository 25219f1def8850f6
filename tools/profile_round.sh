# Round profiles on the GPU box (run from the repo root through gpurun):
#   bench.py tools/profile_round.sh ROUND TAG [bench args...]
#   the bench line, rocprofv3 kernel-trace stats of the same command, and the two HBM counter passes of plan_kernel
#   (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950) in the benched configuration: one plan_kernel dispatch
#   holds the leader, its scouts and its helpers (round 5), so serialised dispatches change nothing.  Outputs under
#   gpurun_out/ROUND_TAG_* (merged back by gpurun); then, locally: tools/rocpd_summary.py stats / pmc on the merged .db
#   files -> profiles/ROUND_TAG_kernel_stats.txt and profiles/ROUND_pmc_TAG.json (read by bench.py for this workload).
set -e
ROUND=${1:-r05}
TAG=${2:-c2}
shift 2 || true
R=$PWD
OUT=$R/gpurun_out
P=$OUT/${ROUND}_${TAG}
mkdir -p $OUT
timeout -k 10 600 python bench.py "$@" > ${P}_bench.json 2> ${P}_bench.err
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d ${P}_prof_kt -o kt -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 "$@" > ${P}_kt.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d ${P}_prof_pmc -o pmc -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 "$@" > ${P}_pmc.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d ${P}_prof_pmcw -o pmcw -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 "$@" > ${P}_pmcw.log 2>&1
cd $R
