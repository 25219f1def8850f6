"""Fixed start-up cost of a planning call vs per-iteration cost before the first solution (C2, seed 1001): device
time to finish N iterations for small N (first solution at iteration 60), plus the host-clock call time."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

sc = scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
for n in (0, 1, 2, 5, 10, 20, 40, 59):
    best = None
    for rep in range(4):
        t = time.perf_counter()
        r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=n, seed=1001))
        wall = time.perf_counter() - t
        ms, pms, nl = gp.last_kernel_ms()
        row = (r["time_total"] * 1e3, pms, wall * 1e3)
        best = row if best is None or row[0] < best[0] else best
    print("iterations %3d: device %.3f ms, plan kernel %.3f ms, host call %.3f ms" % ((n,) + best), flush=True)
    if n <= 1:
        print("   phases (us):", {k: round(v * 1e6, 1) for k, v in r["phases"].items() if v and not k.startswith(("n_", "checked", "slots"))}, flush=True)
