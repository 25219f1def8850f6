"""Collision-tile latency probe: one workgroup streams tiles of C2 configurations back to back (grid 1), and
the full-chip batch rate (grid = all tiles).  Configurations: points of the edges a C2 planner run checks
(tree nodes -> parents, interpolated), plus uniformly random ones."""
import ctypes
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import _lib as L, scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

# SMP_SCENE=c5: the 2 cm clutter scene (BASELINE configs[4]) instead of C2's box room
sc = scenes.clutter_cloud() if os.environ.get("SMP_SCENE") == "c5" else scenes.box_room()
print("scene %s: %d occupied keys" % (sc.name, len(sc.keys)), flush=True)
gp = GpuPlanner(path_optimality_threshold=-math.inf)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
print("scene set", flush=True)
r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=1500, seed=1))
print("planned %d iterations" % r["iterations"], flush=True)
qs = []
for w in (0, 1):
    par, conf, _ = gp.tree(w)
    for i in range(1, len(par)):
        p = par[i]
        for s in range(21):
            qs.append(conf[p] + s * (conf[i] - conf[p]) / 20.0)
Q = np.array(qs)
rng = np.random.default_rng(0)
R = np.column_stack([rng.uniform(-5, 5, len(Q)), rng.uniform(-5, 5, len(Q))] +
                    [rng.uniform(-2, 2, len(Q)) for _ in range(6)])
# planner-like expand edges: from a random tree node one step (0.5) towards a uniform sample, 21 points each -- the
# configurations the planner's collision jobs check (new edges, often near or into obstacles)
from oracle import oracle as O  # noqa: E402  (joint limits of the model; test infrastructure, not the path measured)
orob = O.OracleRobot(L.MODEL_JSON)
nodes = np.concatenate([gp.tree(w)[1] for w in (0, 1)])
E = []
while len(E) * 21 < len(Q):
    a = nodes[rng.integers(len(nodes))]
    x = np.concatenate([[rng.uniform(*sc.env_x), rng.uniform(*sc.env_y)],
                        [rng.uniform(orob.q_min[j], orob.q_max[j]) for j in range(2, 8)]])
    d = np.linalg.norm(x - a)
    b = a + (x - a) * (0.5 / d) if d > 0.5 else x
    E.append(a + np.linspace(0.0, 1.0, 21)[:, None] * (b - a)[None, :])
P = np.concatenate(E)
# connect-like edges (the leader's connect near loop): a node of one tree to a node of the other within the near
# radius (4.0), 21 points each -- long edges, often through obstacles
t0, t1 = gp.tree(0)[1], gp.tree(1)[1]
K = []
while len(K) * 21 < len(Q):
    a = t0[rng.integers(len(t0))]
    b = t1[rng.integers(len(t1))]
    if np.linalg.norm(b - a) < 4.0:
        K.append(a + np.linspace(0.0, 1.0, 21)[:, None] * (b - a)[None, :])
K = np.concatenate(K)
lib = L.lib()
sets = {"tree-edges": Q, "expand-edges": P, "connect-edges": K, "random": R}
for name in os.environ.get("SMP_SETS", "tree-edges,expand-edges,connect-edges,random").split(","):
    X = sets[name]
    soa = np.ascontiguousarray(X.T)
    n = len(X)
    # tile < 0: the helpers' job tiles (collide_wide, -tile configurations spread over the workgroup)
    shapes = [(int(v), 1) for v in os.environ.get("SMP_TILES", "8,-8,-4,-2,-1").split(",")] + [(32, 2048), (-1, 2048)]
    for tile, grid in shapes:
        ms = ctypes.c_double()
        hz = ctypes.c_double()
        ticks = (ctypes.c_uint64 * 12)()
        L.check(lib.smp_probe_check_latency(gp.h, soa.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n, 1, 1, grid, tile,
                                            ctypes.byref(ms), ticks, ctypes.byref(hz)))
        ct = abs(tile)
        tiles = (n + ct - 1) // ct
        per_tile_us = [t / hz.value * 1e6 / (tiles if grid == 1 else max(1, tiles // grid)) for t in ticks]
        print("%-10s tile %2d n %7d grid %5d: %.2f ms  %.3g configs/s  per tile %.2f us  stages(us) A %.2f B %.2f C0 %.2f C %.2f"
              % (name, tile, n, grid, ms.value, n / (ms.value * 1e-3), ms.value * 1e3 / tiles * (grid if grid > 1 else 1) /
                 (1 if grid == 1 else min(grid, tiles)), *per_tile_us[:4]), flush=True)
        if tile > 0:
            print("   shader clock %.3f GHz; wave 0 in C: centres + map sweeps %.2f us, self test %.2f us per tile" % (
                ticks[4] / (ticks[5] / hz.value) / 1e9 if ticks[5] else 0, per_tile_us[6], per_tile_us[7]), flush=True)
        else:
            print("   shader clock %.3f GHz; wave 0: primitive sweeps %.2f us, sphere sweeps %.2f us, self %.2f us per "
                  "tile" % (ticks[4] / (ticks[5] / hz.value) / 1e9 if ticks[5] else 0, *per_tile_us[6:9]), flush=True)
