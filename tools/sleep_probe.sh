# Helper poll interval probe: the SMP_JOB_PROF planner phase report (C2, 4203 iterations) for library builds given as
# arguments (e.g. SMP_HELPER_SLEEP variants), then helpers at 200 / 64 / 16 with the first; outputs under gpurun_out/
set -e
mkdir -p gpurun_out
: > gpurun_out/sleep_probe.log
for lib in "$@"; do
  echo "== $lib" >> gpurun_out/sleep_probe.log
  SMP_JOB_PROF=1 SMP_LIB=$lib timeout -k 10 120 python tools/perf_probe.py 4203 >> gpurun_out/sleep_probe.log 2>&1
done
for h in 64 16; do
  echo "== $1 helpers $h" >> gpurun_out/sleep_probe.log
  SMP_HELPERS=$h SMP_JOB_PROF=1 SMP_LIB=$1 timeout -k 10 120 python tools/perf_probe.py 4203 >> gpurun_out/sleep_probe.log 2>&1
done
