"""Per-query view of a many-query step (bench.py --workload c3 / c5): the batch's kernel time and launches, then each
query's iterations, checks and tree sizes, and (SMP_ALONE=1) each query planned alone with the batch's helper count.
Usage: SMP_SCENE=c5 python tools/batch_probe.py [queries] [samples]"""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

nq = int(sys.argv[1]) if len(sys.argv) > 1 else 8
samples = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
sc = scenes.clutter_cloud() if os.environ.get("SMP_SCENE", "c5") == "c5" else scenes.box_room()
print("scene %s, %d queries, %d samples each" % (sc.name, nq, samples), flush=True)
gp = GpuPlanner(path_optimality_threshold=-math.inf, scout=int(os.environ.get("SMP_SCOUT", "1")))
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
pairs = scenes.random_queries(sc, nq, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))
sel = [int(v) for v in os.environ.get("SMP_QSEL", "").split(",") if v]  # a subset of the queries (same ids)
ids = sel or list(range(nq))


def queries(seed):
    return [GpuPlanner.make_query(pairs[k][0], pairs[k][1], sc.env_x, sc.env_y, seed=seed, query_id=k,
                                  samples=samples) for k in ids]


gp.plan_batch(queries(0))  # warmup (the bench's step -1 uses seed 0)
t = time.perf_counter()
rs = gp.plan_batch(queries(1))
dt = time.perf_counter() - t
ms, pms, nl = gp.last_kernel_ms()
tot = sum(r["configs_checked"] for r in rs)
print("batch: wall %.3f s, plan kernels %.3f s, launches %d, %.0f configs/s, helpers %d scout %d" % (
    dt, pms / 1e3, nl, tot / dt, rs[0]["helpers"], rs[0]["scout"]), flush=True)
for k, r in zip(ids, rs):
    print("  q%d: iters %6d checked %7d nodes %5d/%5d first_iter %5d nn %d" % (
        k, r["iterations"], r["configs_checked"], r["nodes_start"], r["nodes_goal"], r["first_solution_iter"],
        r["nn_nodes_scanned"]), flush=True)
if os.environ.get("SMP_ORACLE"):  # each query's oracle run (test infrastructure: the checker, never the product)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle as O
    orc = O.Oracle(O.OracleRobot(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                              "squirrel_motion_planner_amd", "data", "robotino_model.json")),
                   O.OracleScene(sc.keys, sc.res))
    for k, r in zip(ids, rs):
        s, g = pairs[k]
        o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, seed=1, query=k, opt_thresh=-math.inf, threads=1,
                     max_checked=samples, max_iter=0)
        same = o["iterations"] == r["iterations"] and o["checked"] == r["configs_checked"]
        print("  oracle q%d: iters %6d checked %7d nodes %5d/%5d %s" % (
            k, o["iterations"], o["checked"], o["n_start"], o["n_goal"], "same" if same else "DIFFERENT"), flush=True)
if os.environ.get("SMP_ALONE"):
    h = rs[0]["helpers"]
    ga = GpuPlanner(path_optimality_threshold=-math.inf, helpers=h, scout=max(rs[0]["scout"], 1))
    ga.set_scene(Scene.from_keys(sc.keys, sc.res))
    for k, q in zip(ids, queries(1)):
        t = time.perf_counter()
        r = ga.plan(q)
        dt = time.perf_counter() - t
        print("  alone q%d (%d helpers): %.3f s, %.1f us/iter, %.0f configs/s" % (
            k, h, dt, dt * 1e6 / max(r["iterations"], 1), r["configs_checked"] / dt), flush=True)
