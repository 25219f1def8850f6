# bench.py (C2, no CPU leg) for helper-workgroup caps and the leader's share of them; outputs under gpurun_out/
set -e
mkdir -p gpurun_out
for c in 200 230 245; do for dv in 2 3 4; do
  echo "cap $c lead_div $dv: $(SMP_HELPER_CAP=$c SMP_LEAD_DIV=$dv timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f configs/s ttff %.3f ms helpers %s" % (d["value"], d["time_to_first_feasible_path_s"]*1e3, d["config"]["helpers_per_query"]))')"
done; done
