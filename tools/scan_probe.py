"""Where a distributed tree scan's time goes (SMP_SCAN_PROF build): C2 seed 1 at growing iteration budgets; per scan
the write-back + publication, the publisher's own slice, the collection of the helpers' slices and the merge, and per
helper slice its pickup, acquire and slice clocks (device clock, 100 MHz).

  make -C squirrel_motion_planner_amd EXTRA=-DSMP_SCAN_PROF BUILD=build_sp OUT=lib/libsmp_gpu_sp.so
  SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_sp.so python tools/scan_probe.py 100000 200000
"""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import _lib as L, scenes  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene  # noqa: E402

lib = L.lib()
lib.smp_debug_scanprof.restype = ctypes.c_int
lib.smp_debug_scanprof.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
sc = scenes.box_room()
gp = GpuPlanner(path_optimality_threshold=-math.inf)
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
buf = (ctypes.c_uint64 * 24)()
for iters in [int(v) for v in (sys.argv[1:] or ["100000"])]:
    lib.smp_debug_scanprof(buf, 1)  # reset
    r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=iters, seed=1))
    _, pms, _ = gp.last_kernel_ms()
    if lib.smp_debug_scanprof(buf, 1) != 0:
        sys.exit("not an SMP_SCAN_PROF build")
    v = [int(x) for x in buf]
    n, nh, nn = max(v[0], 1), max(v[7], 1), max(v[12], 1)
    us = lambda t, d: t / 100.0 / d  # noqa: E731
    print("iters %d: %.1f us/iter, nodes %d/%d, %d scans (%d near), %.2f scans/iter, mean participants %.1f, "
          "mean nodes %.0f" % (iters, pms * 1e3 / iters, r["nodes_start"], r["nodes_goal"], v[0], v[12], v[0] / iters,
                               v[14] / n, v[15] / n), flush=True)
    print("   per scan (us): write-back+publish %.2f, own slice %.2f, collection %.2f (near %.2f), merge %.2f; "
          "%.2f rounds, %.3f steals" % (us(v[1], n), us(v[2], n), us(v[3], n), us(v[13], nn), us(v[4], n),
                                        v[6] / n, v[5] / n), flush=True)
    print("   per helper slice (us): pickup %.2f, acquire %.2f, slice %.2f, publication->result %.2f (%d slices)" % (
        us(v[8], nh), us(v[9], nh), us(v[10], nh), us(v[11], nh), v[7]), flush=True)
    nf = max(v[0] - v[12], 1)
    print("   near scans: own slice %.2f, collection %.2f, merge %.2f, helper slice %.2f | nearest scans: own slice %.2f, "
          "collection %.2f, merge %.2f" % (us(v[16], nn), us(v[13], nn), us(v[17], nn), us(v[19], max(v[18], 1)),
                                           us(v[2] - v[16], nf), us(v[3] - v[13], nf), us(v[4] - v[17], nf)), flush=True)
