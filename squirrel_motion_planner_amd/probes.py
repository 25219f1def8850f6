"""Kernel-level probes of libsmp_gpu.so (tests and tools/): not part of the planner API.

tree_scan: the planner's two tree scans run alone in one workgroup (near_probe_kernel, smp_kernels.hip):
find_nearest_neighbour_interpolation and find_near_vertices_interpolation (birrt_star.cpp:4076-4133,
4272-4324) of m query configurations against one tree.
"""
import ctypes

import numpy as np

from . import _lib as L


def _reps_code(reps, slices, fused, inline=False):
    """near_probe_kernel's mode in the sign and high bits of its repetition count: 0 nearest + near_set, 1 the slice
    functions, 2 the fused near_set<20, true>, 3 the fused slice_near<true>, 4 / 5 the helpers' inlined slice forms of
    1 / 3."""
    mode = (4 if fused else 3) + 1 if (slices and inline) else (1 if slices else 0) + (2 if fused else 0)
    return reps if mode == 0 else -(reps + ((mode - 1) << 20))


def tree_scan(q, cost, queries, excl, r, reps=1, device=0, slices=False, fused=False, inline=False):
    """q (n, 8) node configurations, cost (n,) total costs, queries (m, 8), excl (m,) node id left out of the near
    set (-1: none).  Returns nearest ids, near counts, the first / last 20 near ids (ascending (cost, id); -1
    padded) and the device seconds of all nearest / near_set calls."""
    q = np.ascontiguousarray(np.asarray(q, np.float64).T)
    cost = np.ascontiguousarray(cost, np.float64)
    queries = np.ascontiguousarray(queries, np.float64)
    excl = np.ascontiguousarray(excl, np.int32)
    n, m = q.shape[1], queries.shape[0]
    nn = np.zeros(m, np.int32)
    nk = np.zeros(m, np.int32)
    lo = np.zeros((m, 20), np.int32)
    hi = np.zeros((m, 20), np.int32)
    ticks = (ctypes.c_uint64 * 14)()
    hz = ctypes.c_double()
    pd = ctypes.POINTER(ctypes.c_double)
    L.check(L.lib().smp_probe_near(device, q.ctypes.data_as(pd), cost.ctypes.data_as(pd), n, queries.ctypes.data_as(pd),
                                   excl.ctypes.data_as(ctypes.c_void_p), m, float(r), _reps_code(reps, slices, fused, inline),
                                   nn.ctypes.data_as(ctypes.c_void_p), nk.ctypes.data_as(ctypes.c_void_p),
                                   lo.ctypes.data_as(ctypes.c_void_p), hi.ctypes.data_as(ctypes.c_void_p), ticks,
                                   ctypes.byref(hz)), "smp_probe_near")
    return {"nearest": nn, "k": nk, "lo": lo, "hi": hi,
            "t_nearest": ticks[0] / hz.value, "t_near": ticks[1] / hz.value,
            "prof": [ticks[2 + k] for k in range(12)], "clock_hz": hz.value}
