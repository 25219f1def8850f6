"""Finds the first iteration at which a GPU run departs from the oracle (bisection on the iteration budget) for the
C5 bench share's queries (or C3's with argv[1] == 'c3'): prints per query whether the full run matches, and for the
first mismatching one the smallest iteration budget whose counters differ."""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "c5"
samples = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
sc = scenes.clutter_cloud() if which == "c5" else scenes.box_room()
gs = Scene.from_keys(sc.keys, sc.res)
gp = GpuPlanner(path_optimality_threshold=-math.inf)
gp.set_scene(gs)
orob = O.OracleRobot(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "squirrel_motion_planner_amd",
                                  "data", "robotino_model.json"))
orc = O.Oracle(orob, O.OracleScene(sc.keys, sc.res))
pairs = scenes.random_queries(sc, 8, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))
keys = (("iterations", "iterations"), ("configs_checked", "checked"), ("nodes_start", "n_start"), ("nodes_goal", "n_goal"))


def same(r, o):
    return all(r[a] == o[b] for a, b in keys)


qs = [GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, samples=samples, seed=1, query_id=k) for k, (s, g) in enumerate(pairs)]
rs = gp.plan_batch(qs)
bad = None
for k, ((s, g), r) in enumerate(zip(pairs, rs)):
    o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_checked=samples, seed=1, query=k, opt_thresh=-np.inf)
    ok = same(r, o)
    print("query %d: gpu iters %d checked %d nodes %d/%d | oracle %d %d %d/%d  %s" % (
        k, r["iterations"], r["configs_checked"], r["nodes_start"], r["nodes_goal"], o["iterations"], o["checked"],
        o["n_start"], o["n_goal"], "ok" if ok else "DIFFERENT"), flush=True)
    if not ok and bad is None:
        bad = k
if bad is None:
    sys.exit(0)
s, g = pairs[bad]
lo, hi = 0, rs[bad]["iterations"]
while hi - lo > 1:
    mid = (lo + hi) // 2
    r = gp.plan(GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, iterations=mid, seed=1, query_id=bad))
    o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_iter=mid, seed=1, query=bad, opt_thresh=-np.inf)
    if same(r, o):
        lo = mid
    else:
        hi = mid
print("query %d: first differing budget %d iterations" % (bad, hi), flush=True)
for it in (hi - 1, hi):
    r = gp.plan(GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, iterations=it, seed=1, query_id=bad))
    o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_iter=it, seed=1, query=bad, opt_thresh=-np.inf)
    print("  budget %d: gpu checked %d nodes %d/%d | oracle checked %d nodes %d/%d" % (
        it, r["configs_checked"], r["nodes_start"], r["nodes_goal"], o["checked"], o["n_start"], o["n_goal"]), flush=True)
    if it == hi:
        for t in (0, 1):
            par, conf, _ = gp.tree(t)
            op, oc = o["start_parent" if t == 0 else "goal_parent"], o["start_conf" if t == 0 else "goal_conf"]
            n = min(len(par), len(op))
            d = np.nonzero((par[:n] != op[:n]) | np.any(conf[:n] != oc[:n], axis=1))[0]
            print("  tree %d: gpu %d nodes, oracle %d, first differing node %s" % (t, len(par), len(op), d[:3]), flush=True)
