# Early asks (iteration k + 2 asked as soon as its scout is free, rebuilt when its tree is rewired), as the variant
# library lib/libsmp_gpu_early.so (sources squirrel_motion_planner_amd/csrc_early): parity + timing against the build.
set -e
OUT=gpurun_out
mkdir -p $OUT
E=squirrel_motion_planner_amd/lib/libsmp_gpu_early.so
SMP_LIB=$E timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_errors.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/parity_early.log 2>&1
SMP_LIB=$E timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_early.txt 2>&1
timeout -k 10 120 python -u tools/perf_probe.py 4000 > $OUT/perf_probe_base2.txt 2>&1
SMP_LIB=$E timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_early.json 2> $OUT/bench_early.err
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_base2.json 2> $OUT/bench_base2.err
SMP_TRACE_W0=16 SMP_TRACE_NW=6 SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_early_trace.so timeout -k 10 120 python -u tools/trace_probe.py > $OUT/trace_probe_early.txt 2>&1
