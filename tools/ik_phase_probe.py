#!/usr/bin/env python3
"""Per-phase cycles of one IK controller iteration (block 0, s_memtime) from the profiling build:

  make -C squirrel_motion_planner_amd EXTRA=-DSMP_IK_PROF BUILD=build_ikprof OUT=lib/libsmp_gpu_ikprof.so
  SMP_LIB=squirrel_motion_planner_amd/lib/libsmp_gpu_ikprof.so python tools/ik_phase_probe.py
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import _lib as L  # noqa: E402
from squirrel_motion_planner_amd.planner import GpuPlanner, Robot  # noqa: E402

lib = L.lib()
lib.smp_probe_ik_prof.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
gp = GpuPlanner(Robot())
buf = (ctypes.c_uint64 * 8)()
ee = [0.5, 0.5, 2.5, 0.0, 0.0, 0.0]  # out of reach: every run takes 1000 iterations
for n in (1, 17, 272):
    q0 = np.tile([0.0, 0.0, 0.99, -1.2, 1.1, 0.0, 0.7, -1.5], (n, 1))
    gp.ik_solve([ee], q0)
    lib.smp_probe_ik_prof(buf)
    r = gp.ik_solve([ee], q0)
    ms = gp.last_kernel_ms()[0]
    lib.smp_probe_ik_prof(buf)
    it = max(buf[6], 1)
    names = ["jacobian+error", "JJt", "gauss-jordan", "manip", "qdot+update", "fk"]
    tot = sum(buf[i] for i in range(6)) / it
    print("n %4d: kernel %.2f ms, %.2f us/iter; cycles/iter %.0f: %s" % (
        n, ms, ms * 1e3 / int(r["iterations"].max()), tot,
        ", ".join("%s %.0f" % (names[i], buf[i] / it) for i in range(6))), flush=True)
