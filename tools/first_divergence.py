"""Parity hunt: the first iteration budget at which a GPU run (given helpers / scouts) and the oracle disagree on the
counters, for one query (scenes.random_queries seed 7).  Usage: SMP_SCENE=c5 python tools/first_divergence.py QUERY
MAX_ITERS HELPERS SCOUT.  Test infrastructure: the oracle is the checker here."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

k, top, h, ns = (int(a) for a in sys.argv[1:5])
sc = scenes.clutter_cloud() if os.environ.get("SMP_SCENE", "c5") == "c5" else scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf, helpers=h, scout=ns)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
s, g = scenes.random_queries(sc, k + 1, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))[k]
orc = O.Oracle(O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")),
               O.OracleScene(sc.keys, sc.res))
KEYS = (("configs_checked", "checked"), ("nodes_start", "n_start"), ("nodes_goal", "n_goal"),
        ("rewires_start", "rewires_start"), ("rewires_goal", "rewires_goal"), ("first_solution_iter", "first_iter"))


def differs(b):
    r = gp.plan(GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, iterations=b, seed=1, query_id=k))
    o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, seed=1, query=k, opt_thresh=-math.inf, max_iter=b)
    d = ["%s %d/%d" % (kr, r[kr], o[ko]) for kr, ko in KEYS if r[kr] != o[ko]]
    return d, r, o


lo, hi = 0, top  # lo: known same, hi: known different
d, _, _ = differs(hi)
if not d:
    print("same at %d" % hi)
    sys.exit(0)
while hi - lo > 1:
    mid = (lo + hi) // 2
    d, _, _ = differs(mid)
    print("  %d: %s" % (mid, "; ".join(d) or "same"), flush=True)
    if d:
        hi = mid
    else:
        lo = mid
d, r, o = differs(hi)
print("first differing budget %d: %s" % (hi, "; ".join(d)), flush=True)
for kr, ko in KEYS:
    print("   %s gpu %d oracle %d" % (kr, r[kr], o[ko]))
