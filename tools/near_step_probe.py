"""Step times of the fp32-prefiltered near-set slice (slice_near_hist, the form the planner runs from 2048 nodes and in
every distributed-scan slice) on the trees of a C2 planner run and on synthetic uniform trees: thread 0's shader-clock
ticks per step (near_probe_inl_kernel, mode 4), microseconds per call."""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import probes, scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

STEPS = ("scan", "minmax", "hist|direct", "prefix", "gather", "rank", "nn")


def report(label, q, cost, queries, excl, r, reps=10):
    g = probes.tree_scan(q, cost, queries, excl, r, reps=reps, slices=True, inline=True)
    calls = len(queries) * reps
    pf = g["prof"]
    sclk = pf[10] / (pf[11] / g["clock_hz"])
    steps = " ".join("%s %.2f" % (n, pf[k] / sclk / calls * 1e6) for k, n in enumerate(STEPS))
    print("%-22s n %7d mean k %7.0f: %.2f us per call | %s | chunks direct %d hist %d" % (
        label, len(q), g["k"].mean(), g["t_near"] / calls * 1e6, steps, pf[7], pf[8]), flush=True)


iters = [int(v) for v in (sys.argv[1:] or ["4653", "30000"])]
sc = scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
rng = np.random.default_rng(0)
for it in iters:
    gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=it, seed=1))
    par, conf, cost = gp.tree(0)
    m = 32
    idx = rng.integers(0, len(conf), m)
    queries = conf[idx] + rng.normal(0, 0.3, (m, 8))
    for n in sorted({min(len(conf), v) for v in (2048, 4096, 8192, 16384, len(conf))}):
        report("C2 tree @%d it" % it, conf[:n], cost[:n, 0], queries, np.minimum(idx, n - 1), 4.0)
lo = np.array([-5.0, -5.0, -np.pi, -2.9, -1.8, -2.9, -2.2, -2.9])
for n in (4096, 16384, 65536):
    q = rng.uniform(lo, -lo, (n, 8))
    cost = np.sort(rng.uniform(0, 30, n)) + rng.uniform(0, 2, n)
    queries = rng.uniform(lo, -lo, (32, 8))
    report("uniform", q, cost, queries, rng.integers(0, n, 32).astype(np.int32), 4.0)
