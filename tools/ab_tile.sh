# A/B of collision-tile library builds (run from the repo root through gpurun): tile latency probe, then the
# C2 / C3 bench (no CPU leg) for each library given as an argument.  Outputs under gpurun_out/.
set -e
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  SMP_LIB=$lib timeout -k 10 200 python tools/tile_probe.py
done > gpurun_out/tile_ab.log 2>&1
bash tools/lib_sweep.sh "$@"
