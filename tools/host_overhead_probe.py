"""Host side of time to first feasible path (C2, bench seeds): smp_plan entry -> each host stage of the first launch
(SMP_HOST_PROF stamps on stderr), and host-clock vs device-clock TTFF per seed."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

sc = scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
for rep in range(2):
    for seed in (1, 1001, 2001, 3001, 4001):
        r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=200, seed=seed))
        print("rep %d seed %5d: first iter %d, ttff host %.3f ms device %.3f ms (host - device %.3f ms)" % (
            rep, seed, r["first_solution_iter"], r["time_first_solution_host"] * 1e3, r["time_first_solution"] * 1e3,
            (r["time_first_solution_host"] - r["time_first_solution"]) * 1e3), flush=True)
        sys.stderr.flush()
