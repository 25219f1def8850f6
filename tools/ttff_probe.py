"""Time to first feasible path on C2 (bench seeds) for several scout counts: device clocks from the planning
start, leader phase times per pre-solution iteration, and the CPU oracle's time for the same seeds."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

sc = scenes.box_room()
counts = [int(v) for v in (sys.argv[1:] or ["2", "4", "6", "8"])]
for ns in counts:
    gp = GpuPlanner(path_optimality_threshold=-math.inf, scout=ns)
    gp.set_scene(Scene.from_keys(sc.keys, sc.res))
    for seed in (1, 1001, 2001):
        best = None
        for rep in range(3):
            r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=150, seed=seed))
            t = r["time_first_solution"]
            best = t if best is None else min(best, t)
        n = max(r["first_solution_iter"], 1)
        raw = r["phase_raw"]
        print("scouts %d seed %d: first solution iter %d, ttff %.3f ms (best of 3), %.1f us/iter to it | "
              "pre-solution commits %d, no record %d, newer nearest %d, connect completed %d | leader waited %.1f us/iter "
              "(150 iters)" % (r["scout"], seed, r["first_solution_iter"], best * 1e3, best * 1e6 / n,
                               raw[28], raw[29], raw[30], raw[31], r["scout_wait_seconds"] * 1e6 / 150), flush=True)
