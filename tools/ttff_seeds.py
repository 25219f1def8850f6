#!/usr/bin/env python3
"""Time to first feasible path on C2 for the bench's 20 step seeds (1, 1001, ..., 19001): the GPU on the host clock
from smp_plan entry (median of `reps` runs per seed) beside the CPU oracle's from run() entry (one thread, median of
`reps` runs), per seed; how many seeds the GPU is earlier on.  Knobs of the provisioning come from the environment
(SMP_PRE_HELPERS, SMP_LEAD_DIV, SMP_PRE_DELAY, ...; SMP_SCOUT: the scout count).

  python tools/ttff_seeds.py [reps] [out.json]
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402  (the CPU leg: test infrastructure, timed beside the GPU)
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
out = sys.argv[2] if len(sys.argv) > 2 else None
sc = scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf, scout=int(os.environ.get("SMP_SCOUT", "1")))
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
orc = O.Oracle(O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")),
               O.OracleScene(sc.keys, sc.res))
gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=50, seed=99))  # warm-up
rows = []
for k in range(20):
    seed = 1 + 1000 * k
    g, c = [], []
    for _ in range(reps):
        r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=600, seed=seed))
        g.append(r["time_first_solution_host"] if r["time_first_solution_host"] >= 0 else float("nan"))
        o = orc.plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, seed=seed, query=0, opt_thresh=-math.inf,
                     max_iter=600)
        c.append(o["t_first"] if o["t_first"] >= 0 else float("nan"))
    rows.append({"seed": seed, "first_iter": r["first_solution_iter"], "gpu_ms": float(np.median(g)) * 1e3,
                 "cpu_ms": float(np.median(c)) * 1e3, "gpu_runs_ms": [x * 1e3 for x in g],
                 "cpu_runs_ms": [x * 1e3 for x in c]})
    print("seed %5d first iter %4d: gpu %.3f ms  cpu %.3f ms  %s" % (
        seed, r["first_solution_iter"], rows[-1]["gpu_ms"], rows[-1]["cpu_ms"],
        "earlier" if rows[-1]["gpu_ms"] < rows[-1]["cpu_ms"] else "LATER"), flush=True)
gm = np.array([x["gpu_ms"] for x in rows])
cm = np.array([x["cpu_ms"] for x in rows])
summ = {"seeds": 20, "gpu_earlier": int((gm < cm).sum()), "gpu_median_ms": float(np.median(gm)),
        "cpu_median_ms": float(np.median(cm)), "ratio_of_medians": float(np.median(gm) / np.median(cm)),
        "env": {k: v for k, v in os.environ.items() if k.startswith("SMP_")}}
print(json.dumps(summ), flush=True)
if out:
    json.dump({"summary": summ, "rows": rows}, open(out, "w"), indent=1)
