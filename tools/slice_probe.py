"""One workgroup's scan of a range, as a distributed scan's participant does it (slice_nn / slice_near) against the local
scans (nearest / near_set) over the same nodes: microseconds per call and equal results.  Synthetic tree: uniform
configurations in the C2 joint box, costs growing with the index plus noise (a planner tree's costs grow with depth)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from squirrel_motion_planner_amd import probes  # noqa: E402

rng = np.random.default_rng(1)
m, reps = 32, 10
for n in [int(v) for v in (sys.argv[1:] or ["1024", "2048", "4096", "8192", "16384"])]:
    lo = np.array([-5.0, -5.0, -np.pi, -2.9, -1.8, -2.9, -2.2, -2.9])
    hi = -lo
    q = rng.uniform(lo, hi, (n, 8))
    cost = np.sort(rng.uniform(0, 30, n)) + rng.uniform(0, 2, n)
    queries = rng.uniform(lo, hi, (m, 8))
    excl = rng.integers(0, n, m).astype(np.int32)
    a = probes.tree_scan(q, cost, queries, excl, 4.0, reps=reps)
    b = probes.tree_scan(q, cost, queries, excl, 4.0, reps=reps, slices=True)
    c = probes.tree_scan(q, cost, queries, excl, 4.0, reps=reps, slices=True, inline=True)
    same = (np.array_equal(a["nearest"], b["nearest"]) and np.array_equal(a["k"], b["k"]) and
            np.array_equal(a["lo"], b["lo"]) and np.array_equal(a["hi"], b["hi"]) and
            all(np.array_equal(a[f], c[f]) for f in ("nearest", "k", "lo", "hi")))
    calls = m * reps
    sclk = a["prof"][10] / (a["prof"][11] / a["clock_hz"]) / 1e9
    print("n %6d (shader clock %.2f GHz, mean near %6.0f): nearest %.2f / slice_nn %.2f / inlined %.2f us, near_set %.2f / "
          "slice_near %.2f / inlined %.2f us, same %s" % (
              n, sclk, a["k"].mean(), a["t_nearest"] / calls * 1e6, b["t_nearest"] / calls * 1e6,
              c["t_nearest"] / calls * 1e6, a["t_near"] / calls * 1e6, b["t_near"] / calls * 1e6,
              c["t_near"] / calls * 1e6, same), flush=True)
    pf = a["prof"]
    if pf[6] + pf[7] > 0:  # SMP_NEAR_PROF build: near_set's barrier-separated steps (register path)
        fast = max(pf[7], 1)
        print("         near_set register path %d / fallback %d; steps (us/call): %s" % (
            pf[7], pf[6], " ".join("%.2f" % (pf[k] / a["clock_hz"] / fast * 1e6) for k in range(5))), flush=True)
