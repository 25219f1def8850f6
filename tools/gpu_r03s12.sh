# Scout count for 8 queries per GPU (C5, C3 share): automatic (2 scouts at 32 CUs per query) vs 3 and 4.
set -e
OUT=gpurun_out
mkdir -p $OUT
for w in c5 c3; do
  for s in 1 3 4; do
    echo "$w scout $s: $(timeout -k 10 300 python bench.py --workload $w --no-cpu --steps 1 --warmup 1 --scout $s 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f configs/s %.0f it/s scouts %s helpers %s" % (d["value"], d["iterations_per_s"], d["config"]["scout"], d["config"]["helpers_per_query"]))')" >> $OUT/scout_sweep_q8.txt
  done
done
