# bench.py C2 and C3 (no CPU leg) with library variants given as arguments; outputs under gpurun_out/
set -e
mkdir -p gpurun_out
for lib in "$@"; do
  for w in c2 c3; do
    echo "$lib $w: $(SMP_LIB=$lib timeout -k 10 200 python bench.py --workload $w --no-cpu --steps 2 --warmup 1 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f configs/s ttff %.3f ms" % (d["value"], d["time_to_first_feasible_path_s"]*1e3))')"
  done
done > gpurun_out/lib_sweep.log 2>&1
