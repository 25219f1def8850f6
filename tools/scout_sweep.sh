# bench.py (C2, no CPU leg) for scout counts and pre-solution start delays; outputs under gpurun_out/
set -e
mkdir -p gpurun_out
for d in 2 3; do for s in 2 3 4 6; do
  echo "pre_delay $d scout $s: $(SMP_PRE_DELAY=$d timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 --scout $s | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f configs/s ttff %.3f ms" % (d["value"], d["time_to_first_feasible_path_s"]*1e3))')"
done; done
