"""Device timeline of the planner (SMP_TRACE build): thread 0 of the leader and of the scouts log (source line,
device clock) records for a window of iterations of the C2 query; this prints, per role, the mean time between
consecutive trace points (keyed by the two source lines) and the raw timeline of two iterations.

  make -C squirrel_motion_planner_amd EXTRA=-DSMP_TRACE BUILD=build_trace OUT=lib/libsmp_gpu_trace.so
  SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_trace.so python tools/trace_probe.py [iterations]
"""
import collections
import ctypes
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import _lib as L, scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3100
lib = L.lib()
lib.smp_debug_tlog.restype = ctypes.c_int
lib.smp_debug_tlog.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_int]
sc = scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf, scout=int(os.environ.get("SMP_SCOUTS", "1")))
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
buf = (ctypes.c_uint64 * (1 << 18))()
lib.smp_debug_tlog(buf, 1 << 18, 1)  # reset
start, goal = sc.start, sc.goal
if os.environ.get("SMP_TRACE_C3Q"):  # one of C3's random queries (bench.py --workload c3) instead of C2's pair
    pairs = scenes.random_queries(sc, 8, seed=7, check=lambda q: bool(gp.check_configs([q])[0]))
    start, goal = pairs[int(os.environ["SMP_TRACE_C3Q"])]
r = gp.plan(GpuPlanner.make_query(start, goal, sc.env_x, sc.env_y, iterations=iters, seed=1,
                                  query_id=int(os.environ.get("SMP_TRACE_C3Q", "0"))))
n = lib.smp_debug_tlog(buf, 1 << 18, 1)
print("iterations %d, checked %d, first solution iter %d, %d trace records" % (
    r["iterations"], r["configs_checked"], r["first_solution_iter"], n))
a = np.ctypeslib.as_array(buf).astype(np.uint64)
a = a[a != 0]
role = (a >> np.uint64(62)).astype(int)
it = ((a >> np.uint64(54)) & np.uint64(0xff)).astype(int)
line = ((a >> np.uint64(40)) & np.uint64(0x3fff)).astype(int)
clk = (a & np.uint64(0xffffffffff)).astype(np.int64)
TICK_US = 0.01  # wall clock 100 MHz
src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "squirrel_motion_planner_amd",
                        "csrc", "smp_kernels.hip")).read().split("\n")


def func_of(ln):
    for k in range(ln - 1, -1, -1):
        t = src[k]
        if t.startswith("__device__") or t.startswith("__global__"):
            name = t.split("(")[0].split()[-1]
            return name
    return "?"


for rl in sorted(set(role.tolist())):
    m = role == rl
    order = np.argsort(clk[m], kind="stable")
    R_it, R_ln, R_ck = it[m][order], line[m][order], clk[m][order]
    trans = collections.OrderedDict()
    its = sorted(set(R_it.tolist()))
    for k in range(len(R_ck) - 1):
        key = (R_ln[k], R_ln[k + 1])
        d = (R_ck[k + 1] - R_ck[k]) * TICK_US
        s = trans.setdefault(key, [0.0, 0])
        s[0] += d
        s[1] += 1
    tot = (R_ck[-1] - R_ck[0]) * TICK_US
    print("\n=== role %d (%s): %d iterations in window, %.1f us per iteration" % (
        rl, "leader" if rl == 0 else "scout %d" % rl, len(its), tot / max(len(its) - 1, 1)))
    rows = sorted(trans.items(), key=lambda kv: -kv[1][0])
    for (l0, l1), (s, c) in rows[:40]:
        print("  %5.2f us/iter  %6.2f us x %4d   %4d %-22s -> %4d %-22s" % (
            s / max(len(its), 1), s / c, c, l0, func_of(l0)[:22], l1, func_of(l1)[:22]))

# raw timeline of two leader iterations with the scouts' records interleaved
w0 = int(os.environ.get("SMP_TRACE_W0", "20"))
nw = int(os.environ.get("SMP_TRACE_NW", "2"))
sel = (it >= w0) & (it < w0 + nw)
order = np.argsort(clk[sel], kind="stable")
t0 = clk[sel][order][0] if sel.any() else 0
print("\n=== timeline (iterations %d-%d of the window), us from the first record" % (w0, w0 + 1))
for rl_, it_, ln_, ck_ in zip(role[sel][order], it[sel][order], line[sel][order], clk[sel][order]):
    print("  %8.2f  %s it+%d  %4d %s" % ((ck_ - t0) * TICK_US, "L " if rl_ == 0 else "S%d" % rl_, it_ - w0, ln_,
                                         func_of(ln_)))
