"""C5 map-stage probe: the batch checker (smp_check_configs, all CUs, 8-configuration tiles) on the
2 cm clutter scene, for uniformly random configurations and for configurations along short random edges (the
planner's access pattern: neighbouring configurations touch neighbouring cells).  Prints configs/s per set; run it
under rocprofv3 --pmc (tools/c5_counters.sh) for the memory-side bytes and L2 hit rate per configuration."""
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

sc = scenes.clutter_cloud()
gp = GpuPlanner(path_optimality_threshold=-math.inf)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
rng = np.random.default_rng(0)
n = int(os.environ.get("SMP_C5_N", "1000000"))
lo = np.array([sc.env_x[0], sc.env_y[0], -math.pi, -2.9, -1.8, -2.6, -1.6, -2.6])
hi = np.array([sc.env_x[1], sc.env_y[1], math.pi, 2.9, 1.8, 2.6, 1.6, 2.6])
R = rng.uniform(lo, hi, (n, 8))
ne = n // 21
a = rng.uniform(lo, hi, (ne, 8))
b = np.clip(a + rng.normal(0, 0.15, (ne, 8)), lo, hi)
t = np.linspace(0, 1, 21)
E = (a[:, None, :] + t[None, :, None] * (b - a)[:, None, :]).reshape(-1, 8)
for name, X in (("random", R), ("edges", E)):
    gp.check_configs(X[:1000])
    for rep in range(3):
        t0 = time.perf_counter()
        v = gp.check_configs(X)
        ms, _, _ = gp.last_kernel_ms()
        print("%-7s n %8d rep %d: kernel %.2f ms -> %.3g configs/s (wall %.2f s), valid %.3f" % (
            name, len(X), rep, ms, len(X) / (ms * 1e-3), time.perf_counter() - t0, v.mean()), flush=True)
