# Round profiles on the GPU box (run from the repo root through gpurun):
#   bench.py tools/profile_round.sh ROUND TAG [bench args...]
#   the two HBM counter passes of plan_kernel, the bench line, and rocprofv3 kernel-trace stats of the same command
#   (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950) in the benched configuration: one plan_kernel dispatch
#   holds the leader, its scouts and its helpers (round 5), so serialised dispatches change nothing.  Outputs under
#   gpurun_out/ROUND_TAG_* (merged back by gpurun); then, locally: tools/rocpd_summary.py stats / pmc on the merged .db
#   files -> profiles/ROUND_TAG_kernel_stats.txt and profiles/ROUND_pmc_TAG.json (read by bench.py for this workload).
#   The counter passes go first and are summarised on the box into profiles/ there (and gpurun_out/), so the bench
#   line of this same call carries this call's traffic.
set -e
ROUND=${1:-r05}
TAG=${2:-c2}
shift 2 || true
R=$PWD
OUT=$R/gpurun_out
P=$OUT/${ROUND}_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
# SKIP_PMC / SKIP_BENCH / SKIP_KT=1 leave a step out (a long run's steps can go to separate calls)
if [ -z "$SKIP_PMC" ]; then
  cd /tmp
  timeout -k 10 ${PMC_LIMIT:-1000} rocprofv3 --pmc FETCH_SIZE -d ${P}_prof_pmc -o pmc -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 "$@" > ${P}_pmc.log 2>&1
  timeout -k 10 ${PMC_LIMIT:-1000} rocprofv3 --pmc WRITE_SIZE -d ${P}_prof_pmcw -o pmcw -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 "$@" > ${P}_pmcw.log 2>&1
  cd $R
  python3 tools/rocpd_summary.py pmc plan_kernel $R/profiles/${ROUND}_pmc_${TAG}.json ${P}_prof_pmc/pmc_results.db ${P}_prof_pmcw/pmcw_results.db > ${P}_pmc_summary.txt
  cp $R/profiles/${ROUND}_pmc_${TAG}.json ${P}_pmc.json
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 ${BENCH_LIMIT:-600} python bench.py "$@" > ${P}_bench.json 2> ${P}_bench.err
fi
if [ -z "$SKIP_KT" ]; then
  cd /tmp
  # the traced run prints its own bench line (same steps / warmup as the bench): the kernel trace's mean plan_kernel
  # dispatch and that line's ms_per_step come from one process, so kernel <= step is checkable within it
  timeout -k 10 ${KT_LIMIT:-400} rocprofv3 --kernel-trace --stats -d ${P}_prof_kt -o kt -- python3 $R/bench.py --no-cpu --steps ${KT_STEPS:-20} --warmup ${KT_WARMUP:-5} "$@" > ${P}_kt.log 2>&1
  cd $R
  grep '^{"metric"' ${P}_kt.log > ${P}_kt_bench.json || true
fi
