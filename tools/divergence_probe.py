"""Parity hunt: one query planned alone under several (helpers, scouts) settings, each compared with the oracle's run of
the same budget -- counters, then the first differing node of each tree (insertion order is the oracle's).
Usage: SMP_SCENE=c5 python tools/divergence_probe.py QUERY ITERATIONS [h:s ...]   (QUERY: scenes.random_queries seed 7)
Test infrastructure: the oracle is the checker here."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

k, iters = int(sys.argv[1]), int(sys.argv[2])
settings = [tuple(int(x) for x in a.split(":")) for a in sys.argv[3:]] or [(29, 2), (58, 2), (0, 1)]
sc = scenes.clutter_cloud() if os.environ.get("SMP_SCENE", "c5") == "c5" else scenes.box_room()
g0 = GpuPlanner(path_optimality_threshold=-math.inf)
g0.set_scene(Scene.from_keys(sc.keys, sc.res))
s, g = scenes.random_queries(sc, k + 1, seed=7, check=lambda q: bool(g0.check_configs([q])[0]))[k]
if os.environ.get("SMP_DEL0"):  # experiments: only one planner alive at a time
    del g0
orc = O.Oracle(O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")),
               O.OracleScene(sc.keys, sc.res))
o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, seed=1, query=k, opt_thresh=-math.inf, max_iter=iters)
print("oracle q%d %d iterations: checked %d nodes %d/%d first_iter %d cost %.6f" % (
    k, iters, o["checked"], o["n_start"], o["n_goal"], o["first_iter"], o["cost"][0]), flush=True)


def first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(n):
        if not np.array_equal(a[i], b[i]):
            return i
    return None if len(a) == len(b) else n


for h, ns in settings:
    gp = GpuPlanner(path_optimality_threshold=-math.inf, helpers=h, scout=ns)
    gp.set_scene(Scene.from_keys(sc.keys, sc.res))
    r = gp.plan(GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, iterations=iters, seed=1, query_id=k))
    msg = []
    for kr, ko in (("configs_checked", "checked"), ("nodes_start", "n_start"), ("nodes_goal", "n_goal"),
                   ("first_solution_iter", "first_iter"), ("rewires_start", "rewires_start"),
                   ("rewires_goal", "rewires_goal")):
        if r[kr] != o[ko]:
            msg.append("%s %d != %d" % (kr, r[kr], o[ko]))
    if r["cost_best"] != o["cost"]:
        msg.append("cost %.6f != %.6f" % (r["cost_best"][0], o["cost"][0]))
    for w, name in ((0, "start"), (1, "goal")):
        par, conf, cost = gp.tree(w)
        for lab, a, b in (("parent", par, o[name + "_parent"]), ("conf", conf, o[name + "_conf"]),
                          ("cost", cost, o[name + "_cost"])):
            d = first_diff(a, b)
            if d is not None:
                msg.append("%s tree %s first differs at node %d of %d/%d" % (name, lab, d, len(a), len(b)))
    if os.environ.get("SMP_RING_CHECK"):  # SMP_RING_CHECK build: ring / record samples recomputed by the leader
        raw = r["phase_raw"]
        print("  ring check: %d samples taken, %d differ, first at iteration %d" % (
            round(raw[30]), round(raw[28]), round(raw[29]) - 1), flush=True)
        print("  differing: %d the iteration's uniform sample, %d iteration - 1's, %d iteration + 1's, %d other" % (
            tuple(round(raw[k] * 1e8) for k in (20, 21, 22, 23))), flush=True)
    if os.environ.get("SMP_DUMP"):  # the first nodes of each tree, GPU then oracle
        for w, name in ((0, "start"), (1, "goal")):
            par, conf, cost = gp.tree(w)
            for i in range(min(12, len(par))):
                print("  %s %2d gpu par %3d conf %s | oracle par %3d conf %s" % (
                    name, i, par[i], np.array2string(conf[i], precision=4), o[name + "_parent"][i],
                    np.array2string(o[name + "_conf"][i], precision=4)), flush=True)
    del gp
    print("helpers %d scout %d (used %d/%d): %s" % (h, ns, r["helpers"], r["scout"], "; ".join(msg) or "SAME"),
          flush=True)
