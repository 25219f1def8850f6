"""C5 bench share as one batch (8 queries, 1e6 samples): for every query whose run differs from the oracle, the first
differing node of each tree and the oracle iteration that inserted it (bisection on the oracle's iteration budget)."""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

samples = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
sc = scenes.clutter_cloud()
gp = GpuPlanner(path_optimality_threshold=-math.inf)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
orob = O.OracleRobot(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "squirrel_motion_planner_amd",
                                  "data", "robotino_model.json"))
orc = O.Oracle(orob, O.OracleScene(sc.keys, sc.res))
pairs = scenes.random_queries(sc, 8, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))
first_q = int(sys.argv[2]) if len(sys.argv) > 2 else 3
# the query examined goes first in the batch (smp_get_tree reads query 0's trees); the batch holds the same 8 queries
order = [first_q] + [k for k in range(8) if k != first_q]
qs = [GpuPlanner.make_query(pairs[k][0], pairs[k][1], sc.env_x, sc.env_y, samples=samples, seed=1, query_id=k) for k in order]
rs = gp.plan_batch(qs)
trees = {first_q: [gp.tree(t)[:2] for t in (0, 1)]}
for k, r in zip(order, rs):
    s, g = pairs[k]
    if k != first_q:
        continue
    o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_checked=samples, seed=1, query=k, opt_thresh=-np.inf)
    if r["iterations"] == o["iterations"] and r["configs_checked"] == o["checked"]:
        continue
    print("query %d differs: gpu %d iterations, oracle %d" % (k, r["iterations"], o["iterations"]), flush=True)
    for t in (0, 1):
        par, conf = trees[k][t]
        op, oc = o["start_parent" if t == 0 else "goal_parent"], o["start_conf" if t == 0 else "goal_conf"]
        n = min(len(par), len(op))
        d = np.nonzero((par[:n] != op[:n]) | np.any(conf[:n] != oc[:n], axis=1))[0]
        first = int(d[0]) if len(d) else n
        # oracle iteration that inserted node `first` of tree t: smallest budget whose tree has more than `first` nodes
        lo, hi = 0, o["iterations"]
        while hi - lo > 1:
            mid = (lo + hi) // 2
            om = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_iter=mid, seed=1, query=k, opt_thresh=-np.inf)
            if (om["n_start"] if t == 0 else om["n_goal"]) > first:
                hi = mid
            else:
                lo = mid
        print("  tree %d: gpu %d nodes, oracle %d, first differing node %d (oracle inserts it in iteration %d); "
              "gpu node %s parent %s, oracle node %s parent %s" % (
                  t, len(par), len(op), first, hi - 1, conf[first] if first < len(par) else None,
                  par[first] if first < len(par) else None, oc[first] if first < len(op) else None,
                  op[first] if first < len(op) else None), flush=True)
