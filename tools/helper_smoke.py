"""Small C2 queries with 1 and 3 helper workgroups (diagnostics of the job hand-off)."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

sc = scenes.box_room()
for h in [int(v) for v in (sys.argv[1:] or ["1", "3"])]:
    gp = GpuPlanner(path_optimality_threshold=-math.inf, helpers=h)
    gp.set_scene(Scene.from_keys(sc.keys, sc.res))
    t = time.time()
    try:
        r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=int(os.environ.get("SMP_ITERS", "20")), seed=1))
        print("helpers", h, "status", r["status"], "iters", r["iterations"], "checked", r["configs_checked"],
              "%.2fs" % (time.time() - t), "diag(done, ntiles, claim, seq)", r["phase_raw"][28:32], flush=True)
    except Exception as e:  # noqa: BLE001
        print("helpers", h, "error", e, flush=True)
