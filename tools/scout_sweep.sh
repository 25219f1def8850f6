# bench.py (C2, no CPU leg) for scout counts and pre-solution start delays; outputs under gpurun_out/
set -e
mkdir -p gpurun_out
for sd in "4 3" "4 2" "4 4" "6 3" "6 4" "6 5" "8 4" "8 5" "8 6"; do
  set -- $sd
  echo "scout $1 pre_delay $2: $(SMP_PRE_DELAY=$2 timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 --scout $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f configs/s ttff %.3f ms" % (d["value"], d["time_to_first_feasible_path_s"]*1e3))')"
done
