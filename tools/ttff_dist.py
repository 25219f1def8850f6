#!/usr/bin/env python3
"""Time to first feasible path on C2 (bench seeds), every repetition: device clocks from the planning start.

  SMP_PRE_DELAY=d python tools/ttff_dist.py <scouts> [reps]
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

ns = int(sys.argv[1]) if len(sys.argv) > 1 else 0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
sc = scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf, scout=ns if ns else 1)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
for seed in (1, 1001, 2001):
    ts, det = [], []
    for _ in range(reps):
        r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=150, seed=seed))
        ts.append(r["time_first_solution"] * 1e3)
        raw = r["phase_raw"]
        det.append("%.2f(w%.0f c%d n%d)" % (ts[-1], r["scout_wait_seconds"] * 1e6, raw[28], raw[29]))
    print("scouts %d pre_delay %s seed %d: ttff ms (leader wait us, pre-commits, no record) %s | median %.3f" % (
        r["scout"], os.environ.get("SMP_PRE_DELAY", "-"), seed, " ".join(det), np.median(ts)), flush=True)
