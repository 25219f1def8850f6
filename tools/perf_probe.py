"""Timing probe of the planner kernel at growing iteration budgets (C2) and of the batch check kernel."""
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

# SMP_SCENE=c5: the 2 cm clutter scene and one of C5's random queries (bench.py --workload c5, query SMP_C5Q)
sc = scenes.clutter_cloud() if os.environ.get("SMP_SCENE") == "c5" else scenes.box_room()
print("scene %s" % sc.name, flush=True)
gp = GpuPlanner(path_optimality_threshold=-math.inf, helpers=int(os.environ.get("SMP_HELPERS", "0")),
                scout=int(os.environ.get("SMP_SCOUT", "1")))
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
start, goal = sc.start, sc.goal
if os.environ.get("SMP_C5Q"):  # query k of the bench's random pairs (scenes.random_queries, seed 7)
    k = int(os.environ["SMP_C5Q"])
    start, goal = scenes.random_queries(sc, k + 1, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))[k]
for iters in [int(v) for v in (sys.argv[1:] or ["2000", "10000", "50000"])]:
    t = time.perf_counter()
    r = gp.plan(GpuPlanner.make_query(start, goal, sc.env_x, sc.env_y, iterations=iters, seed=1))
    dt = time.perf_counter() - t
    _, pms, nl = gp.last_kernel_ms()
    print("iters %7d wall %.2fs kernel %.2fs launches %d  us/iter %.1f  checked %d (%.0f/s)  nodes %d/%d "
          "nn %d near %d first_iter %d t_first %.3f cost %.3f" %
          (iters, dt, pms / 1e3, nl, pms * 1e3 / iters, r["configs_checked"], r["configs_checked"] / (pms / 1e3),
           r["nodes_start"], r["nodes_goal"], r["nn_nodes_scanned"], r["near_nodes_scanned"],
           r["first_solution_iter"], r["time_first_solution"], r["cost_best"][0]), flush=True)
    print("   phases:", {k: round(v, 3) for k, v in r["phases"].items()}, flush=True)
    print("   samples precomputed by the run-ahead sampler: %d of %d" % (r["samples_precomputed"], r["iterations"]),
          flush=True)
    print("   helpers %d scout %d: nn hits %d, near hits %d, edge hits %d misses %d, leader waited %.1f us/iter" % (
        r["helpers"], r["scout"], r["scout_nn_hits"], r["scout_near_hits"], r["scout_edge_hits"],
        r["scout_edge_misses"], r["scout_wait_seconds"] * 1e6 / max(r["iterations"], 1)), flush=True)
    sp = r["scout_phases"]
    if sp[30] > 0:
        ns = sp[30]
        print("   scout (us per pass, %d passes): sample %.1f nn %.1f expand %.1f near %.1f choose %.1f via %.1f rewire %.1f"
              " | publish %.1f busy %.1f idle %.1f | edge_costs %.1f tiles(job) %.1f" % (
                  ns, *[sp[k] * 1e6 / ns for k in (0, 1, 2, 3, 4, 5, 6, 29, 31, 28, 9, 7)]), flush=True)
    raw = r["phase_raw"]
    if r["first_solution_iter"] < 0 or r["first_solution_iter"] > 0:
        # the leader's pre_commit outcomes (plain builds: prof[28..31]): record committed / no usable record / a node
        # appended since the record's snapshot is nearer / connect redone in full
        print("   pre_commit outcomes: committed %d, no record %d, newer nearest %d, connect redone %d" % tuple(
            int(v) for v in raw[28:32]), flush=True)
        if sp[26] > 0:  # SMP_PRE_REFRESH=1: scout passes started over on newer tree sizes
            print("   scout passes redone on newer sizes: %d" % int(sp[26]), flush=True)
    nj = max(raw[15] * 1e8, 1)
    print("   jobs %d: publish %.1f us, own %.1f us, wait %.1f us per job" % (
        raw[15] * 1e8, raw[12] * 1e6 / nj, raw[13] * 1e6 / nj, raw[14] * 1e6 / nj), flush=True)
    if os.environ.get("SMP_SAMPLE_PROF"):  # SMP_SAMPLE_PROF build: ellipse sampler stage clocks (ticks, slots 28-30)
        rounds = max(raw[30], 1)
        print("   sample_ellipse: %d rounds, stage 1 %.2f us, stage 2 %.2f us per round" % (
            rounds, raw[28] / 1e2 / rounds, raw[29] / 1e2 / rounds), flush=True)
    if os.environ.get("SMP_JOB_PROF"):  # SMP_JOB_PROF build: helper pickup / tile-finish delay after publication
        n = max(raw[29], 1)
        print("   helpers: %d pickups, pickup %.2f us, tile finished %.2f us after publication (mean)" % (
            raw[29], raw[28] / 1e2 / n, raw[30] / 1e2 / n), flush=True)
        nt = max(r["phases"]["n_tiles"], 1)
        print("   helper tile stages (us per tile, approx.): A %.2f B %.2f C-centres %.2f C %.2f" % tuple(
            raw[12 + i] * 1e6 / nt for i in range(4)), flush=True)
    if os.environ.get("SMP_DETAIL_PROF"):  # SMP_DETAIL_PROF build: serial-section clocks (ticks, slots 28-31)
        print("   serial sections (us/iter): rewire commit %.2f (cost_update %.2f), connect replay %.2f, insert_via %.2f"
              % tuple(raw[k] / 1e2 / iters for k in (28, 29, 30, 31)), flush=True)
    if os.environ.get("SMP_VIA_PROF"):  # SMP_VIA_PROF build: the leader's via_chain_w clocks (ticks, slots 28-31)
        ns = max(r["phases"]["n_via_steps"], 1)
        print("   via chains: %d steps; per step: stepping + edge step %.2f us, segment norms %.2f us, ordered sums %.2f us;"
              " entry %.2f us in all" % (ns, raw[28] / 1e2 / ns, raw[29] / 1e2 / ns, raw[30] / 1e2 / ns,
                                         raw[31] / 1e2), flush=True)
    if os.environ.get("SMP_WAIT_PROF"):  # SMP_WAIT_PROF build: the leader's record waits by stage (ticks, 28-31)
        print("   leader waits (us/iter): nn + expand %.2f, near + choose %.2f, rewire %.2f, connect %.2f" % tuple(
            raw[k] / 1e2 / iters for k in (28, 29, 30, 31)), flush=True)
    if raw[31] > 0 and not any(os.environ.get(v) for v in ("SMP_DETAIL_PROF", "SMP_VIA_PROF", "SMP_WAIT_PROF")):  # SMP_NEAR_PROF build: wave-0 clocks of near_set
        nc = raw[31] * 1e8
        print("   near_set (%d calls, wave 0): scan %.1f us (insert %.1f us), merge %.1f us per call" % (
            nc, raw[28] * 1e6 / nc, raw[29] * 1e6 / nc, raw[30] * 1e6 / nc), flush=True)
rng = np.random.default_rng(0)
n = 2_000_000
q = np.column_stack([rng.uniform(-6, 5, n), rng.uniform(-6, 5, n)] + [rng.uniform(-2, 2, n) for _ in range(6)])
gp.check_configs(q[:1000])
t = time.perf_counter()
v = gp.check_configs(q)
dt = time.perf_counter() - t
ms, _, _ = gp.last_kernel_ms()
print("check_configs: %d configs, kernel %.2f ms -> %.3g configs/s (wall %.2f s), valid %.3f" %
      (n, ms, n / (ms / 1e3), dt, v.mean()))
