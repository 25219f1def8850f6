"""Leader phase times in microseconds per iteration (device clocks) for short C2 runs (pre-solution view)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

sc = scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf, helpers=int(os.environ.get("SMP_HELPERS", "0")))
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
for iters in [int(v) for v in (sys.argv[1:] or ["84", "300"])]:
    r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=iters, seed=1))
    n = max(r["iterations"], 1)
    ph = r["phases"]
    keys = ["sample", "nearest", "expand", "near", "choose_parent", "rewire", "connect", "edge_costs", "via_chains"]
    print("iters %d (first solution at %d, t_first %.3f ms): " % (n, r["first_solution_iter"], r["time_first_solution"] * 1e3)
          + " ".join("%s %.1f" % (k, ph[k] * 1e6 / n) for k in keys)
          + " | leader waited for the scout %.1f us/iter, scout nn hits %d edge hits %d" % (
              r["scout_wait_seconds"] * 1e6 / n, r["scout_nn_hits"], r["scout_edge_hits"]), flush=True)
