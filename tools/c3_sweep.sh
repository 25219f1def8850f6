# C3 share of one GPU (8 queries) for helper counts; outputs under gpurun_out/
set -e
mkdir -p gpurun_out
for h in 8 16 24 0; do
  echo "helpers $h: $(timeout -k 10 200 python bench.py --workload c3 --no-cpu --steps 1 --warmup 1 --helpers $h 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f configs/s ttff %.3f ms helpers %d scout %d" % (d["value"], d["time_to_first_feasible_path_s"]*1e3, d["config"]["helpers_per_query"], d["config"]["scout"]))')"
done > gpurun_out/c3_sweep.log 2>&1
