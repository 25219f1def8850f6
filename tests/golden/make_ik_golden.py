"""Golden IK runs of the CPU oracle (oracle/smp_oracle.cpp ik_solve): tests/golden/ik_golden.npz.

The reference controller (control_laws.cpp run_VDLS_Control_Connector) needs ROS / KDL / Eigen and cannot run
here, so these vectors pin the oracle's restatement against regressions and give the GPU tests fixed inputs:
  * findGoalPose candidate runs for four end-effector goals (hand downward / sideways, reachable, unreachable),
  * goals that are the chain FK of random configurations, started from random configurations,
  * starts at the singular zero arm (manipulability fallback path) and near it (damped path).
Inputs are end-effector poses [x, y, z, roll, pitch, yaw] and start configurations, i.e. what smp_ik_solve takes.

    python tests/golden/make_ik_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

MODEL = os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")


def rpy_of(quat_xyzw):
    from scipy.spatial.transform import Rotation
    return Rotation.from_quat(quat_xyzw).as_euler("xyz")


def random_arm(rng, R, n, base=1.5):
    lo, hi = R.q_min.copy(), R.q_max.copy()
    lo[:2], hi[:2] = -base, base
    return rng.uniform(lo, hi, (n, 8))


def build():
    R = O.OracleRobot(MODEL)
    orc = O.Oracle(R)
    rng = np.random.default_rng(20261016)
    ee_rows, q_rows, kinds = [], [], []
    cur = np.zeros(8)
    goals = [[0.8, 0.3, 0.5, 1.57, 0.0, 0.3],    # sideways hand (tf y axis horizontal)
             [0.6, -0.4, 0.25, 0.0, 1.57, 0.0],  # pitched
             [1.0, 1.0, 0.2, 3.14, 0.0, 0.0],    # downward-ish
             [0.5, 0.5, 2.5, 0.0, 0.0, 0.0]]     # out of reach
    for g in goals:
        t, _ = O.goal_candidates(g, cur, 20.0)
        for row in t:
            ee_rows.append(g)
            q_rows.append(row[19:27])
            kinds.append(0)
    qg = random_arm(rng, R, 24)
    ee, _ = orc.ik_fk_jac(qg)
    for i in range(len(qg)):
        ee_rows.append(list(ee[i, :3]) + list(rpy_of(ee[i, 3:7])))
        q0 = qg[i] + rng.normal(0.0, 0.3, 8)
        q0 = np.clip(q0, R.q_min, R.q_max)
        q_rows.append(q0)
        kinds.append(1)
    for i in range(6):
        g = goals[i % 3]
        q0 = np.zeros(8)
        q0[:2] = rng.uniform(-0.5, 0.5, 2)
        if i >= 3:
            q0[3:] = rng.normal(0.0, 0.02, 5)
        ee_rows.append(g)
        q_rows.append(q0)
        kinds.append(2)
    ee_rows = np.array(ee_rows, np.float64)
    q_rows = np.array(q_rows, np.float64)
    r = orc.ik_solve(O.ik_tasks(ee_rows, q_rows))
    return dict(ee=ee_rows, q_init=q_rows, kind=np.array(kinds, np.int32), q=r["q"], err=r["err"],
                manip=r["manip"], reached=r["reached"], iters=r["iters"], fallback=r["fallback"])


if __name__ == "__main__":
    d = build()
    np.savez_compressed(os.path.join(HERE, "ik_golden.npz"), **d)
    print("%d runs: %d reached, %d fallback runs, iterations %d..%d" % (
        len(d["ee"]), d["reached"].sum(), (d["fallback"] > 0).sum(), d["iters"].min(), d["iters"].max()))
