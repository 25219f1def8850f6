"""Tree-scan timing: nearest and near_set of one workgroup on the trees of a C2 planner run (sizes as the
planner sees them), microseconds per call."""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import probes, scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
cache = sys.argv[2] if len(sys.argv) > 2 else None  # .npz: reuse one tree across library variants (SMP_LIB)
if cache and os.path.exists(cache):
    z = np.load(cache)
    conf, cost = z["conf"], z["cost"]
else:
    sc = scenes.box_room()
    gp = GpuPlanner(path_optimality_threshold=-math.inf)
    gp.set_scene(Scene.from_keys(sc.keys, sc.res))
    gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=iters, seed=1))
    par, conf, cost = gp.tree(0)
    if cache:
        np.savez(cache, conf=conf, cost=cost)
rng = np.random.default_rng(0)
m = 64
idx = rng.integers(0, len(conf), m)
queries = conf[idx] + rng.normal(0, 0.3, (m, 8))
for n in (len(conf) // 4, len(conf) // 2, len(conf)):
    reps = 20
    r = probes.tree_scan(conf[:n], cost[:n, 0], queries, np.minimum(idx, n - 1), 4.0, reps=reps)
    calls = m * reps
    print("n %6d  nearest %.2f us  near_set %.2f us per call  (mean k %.0f)" % (
        n, r["t_nearest"] / calls * 1e6, r["t_near"] / calls * 1e6, r["k"].mean()), flush=True)
    pf = r["prof"]
    if pf[6] + pf[7] > 0:  # SMP_NEAR_PROF build
        fast = max(pf[7], 1)
        print("         register path %d / fallback %d; steps (us/call): scan %s" % (
            pf[7], pf[6], " ".join("%.2f" % (pf[k] / r["clock_hz"] / fast * 1e6) for k in range(5))), flush=True)
