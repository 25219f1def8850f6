"""C3 on one GPU: the 8 random queries as one batch vs each alone with the same helper count; per query the
iterations, checked configurations, phase times per iteration and scout counters."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

sc = scenes.box_room()
nq = int(sys.argv[1]) if len(sys.argv) > 1 else 8
samples = int(sys.argv[2]) if len(sys.argv) > 2 else 300000
gp = GpuPlanner(path_optimality_threshold=-math.inf, helpers=int(os.environ.get("SMP_HELPERS", "0")),
                scout=int(os.environ.get("SMP_SCOUT", "1")))
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
pairs = scenes.random_queries(sc, nq, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))
qs = [GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, samples=samples, seed=1, query_id=i) for i, (s, g) in enumerate(pairs)]
rs = gp.plan_batch(qs)
ms, pms, nl = gp.last_kernel_ms()
h = rs[0]["helpers"]
print("batch of %d: kernel %.1f ms, %d launches, helpers %d scout %d" % (nq, pms, nl, h, rs[0]["scout"]))


def row(r, tag):
    n = max(r["iterations"], 1)
    ph = r["phases"]
    print("  %-8s iters %6d checked %8d (%.0f/iter) t_total %.1f ms -> %.1f us/iter | sample %.1f nn %.1f expand %.1f "
          "near %.1f choose %.1f rewire %.1f connect %.1f | waited %.1f us/iter" % (
              tag, r["iterations"], r["configs_checked"], r["configs_checked"] / n, r["time_total"] * 1e3,
              r["time_total"] * 1e6 / n, *[ph[k] * 1e6 / n for k in ("sample", "nearest", "expand", "near",
                                                                          "choose_parent", "rewire", "connect")],
              r["scout_wait_seconds"] * 1e6 / n), flush=True)
    print("           checked configurations per slot checked (reference-semantics / actual tile slots): " +
          " ".join("%s %.2f" % (k, ph["checked_" + k] / max(ph["slots_" + k], 1))
                   for k in ("expand", "choose", "rewire", "connect")) +
          " | tiles %d" % ph["n_tiles"], flush=True)
    raw = r["phase_raw"]
    nj = max(raw[15] * 1e8, 1)
    print("           jobs %.1f/iter: publish %.1f us, own tiles %.1f us, wait %.1f us per job; tiles/job %.1f" % (
        nj / n, raw[12] * 1e6 / nj, raw[13] * 1e6 / nj, raw[14] * 1e6 / nj, ph["n_tiles"] / nj), flush=True)


for i, r in enumerate(rs):
    row(r, "q%d" % i)
gp1 = GpuPlanner(path_optimality_threshold=-math.inf, helpers=h)
gp1.set_scene(Scene.from_keys(sc.keys, sc.res))
for i in range(min(nq, 3)):
    r = gp1.plan(qs[i])
    row(r, "alone%d" % i)
