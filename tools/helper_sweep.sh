# bench.py (C2, no CPU leg) for helper-workgroup caps and scout counts; outputs under gpurun_out/
set -e
mkdir -p gpurun_out
for c in 127 160 200 250; do for s in 2 4; do
  echo "cap $c scout $s: $(SMP_HELPER_CAP=$c SMP_PRE_DELAY=3 timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 --scout $s | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f configs/s ttff %.3f ms helpers %s" % (d["value"], d["time_to_first_feasible_path_s"]*1e3, d["config"]["helpers_per_query"]))')"
done; done
