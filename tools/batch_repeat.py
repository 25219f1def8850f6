"""Repeats the 4-query C2 batch of test_batch_equals_single (150 iterations each) and counts runs whose batch
results differ from the single-query runs (a race detector)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 150
sc = scenes.box_room()
gp = GpuPlanner()
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
qs = [GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=iters, seed=s, query_id=s) for s in range(4)]
ref = [gp.plan(q)["configs_checked"] for q in qs]
bad = 0
for rep in range(reps):
    b = [r["configs_checked"] for r in gp.plan_batch(qs)]
    if b != ref:
        bad += 1
        print("rep %d: batch %s single %s" % (rep, b, ref), flush=True)
print("%d of %d batches differ (%s, pre_commit %s, pre_delay %s)" % (bad, reps, ref, os.environ.get("SMP_PRE_COMMIT", "1"),
                                                                     os.environ.get("SMP_PRE_DELAY", "2")), flush=True)
