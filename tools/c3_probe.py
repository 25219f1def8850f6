"""C3 share of one GPU (8 random C2-scene queries, 1e6-sample budget each): per-query iterations, tree sizes,
checked configurations, and the leader's phase times -- where multi-query throughput goes."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

nq = int(sys.argv[1]) if len(sys.argv) > 1 else 8
samples = int(float(sys.argv[2])) if len(sys.argv) > 2 else 1000000
helpers = int(sys.argv[3]) if len(sys.argv) > 3 else 0
sc = scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf, helpers=helpers)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
pairs = scenes.random_queries(sc, nq, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))
qs = [GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, seed=1, query_id=k, samples=samples) for k, (s, g) in enumerate(pairs)]
gp.plan_batch(qs)
t = time.perf_counter()
rs = gp.plan_batch(qs)
dt = time.perf_counter() - t
tot = sum(r["configs_checked"] for r in rs)
print("%d queries, %.3f s, %.3g configs/s, helpers %d scout %d" % (nq, dt, tot / dt, rs[0]["helpers"], rs[0]["scout"]))
for k, r in enumerate(rs):
    ph = r["phases"]
    it = max(r["iterations"], 1)
    print("q%-2d it %6d checked %8d (%5.1f/it) nodes %6d/%6d t %.3f s (%.1f us/it) first %d | nn %.1f near %.1f "
          "expand %.1f choose %.1f rewire %.1f connect %.1f us/it | waited %.1f us/it" % (
              k, r["iterations"], r["configs_checked"], r["configs_checked"] / it, r["nodes_start"], r["nodes_goal"],
              r["time_total"], r["time_total"] * 1e6 / it, r["first_solution_iter"], ph["nearest"] * 1e6 / it,
              ph["near"] * 1e6 / it, ph["expand"] * 1e6 / it, ph["choose_parent"] * 1e6 / it, ph["rewire"] * 1e6 / it,
              ph["connect"] * 1e6 / it, r["scout_wait_seconds"] * 1e6 / it))
