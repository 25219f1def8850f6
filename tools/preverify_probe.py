"""SMP_PRE_VERIFY build: C5 bench share (8 queries, batch) with every pre-solution commit recomputed; prints the
verification counters (first mismatch: iteration, kind, block)."""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import _lib as L, scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

lib = L.lib()
lib.smp_debug_preverify.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
which = sys.argv[1] if len(sys.argv) > 1 else "c5"
samples = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
sc = scenes.clutter_cloud() if which == "c5" else scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
pairs = scenes.random_queries(sc, 8, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))
buf = (ctypes.c_uint64 * 4)()
lib.smp_debug_preverify(buf, 1)
qs = [GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, samples=samples, seed=1, query_id=k) for k, (s, g) in enumerate(pairs)]
rs = gp.plan_batch(qs)
lib.smp_debug_preverify(buf, 0)
v = buf[1]
print("checks %d; first mismatch: %s" % (buf[0], "none" if v == 0 else "iteration %d kind %d block %d" % (
    v & 0xffffffffff, (v >> 40) & 0xff, v >> 48)))
for k, r in enumerate(rs):
    print("  q%d iterations %d checked %d first solution %d" % (k, r["iterations"], r["configs_checked"], r["first_solution_iter"]))
