"""CPU tests of the IK goal search restatement: the oracle's VDLS controller
(oracle/smp_oracle.cpp ik_solve, restating control_laws.cpp:3283-3712) checked against independent numpy / scipy
kinematics, the reference's candidate order of findGoalPose (squirrel_8dof_planner.cpp:1129-1201), and the
committed golden runs (tests/golden/make_ik_golden.py).  The reference controller itself needs ROS / KDL / Eigen,
so these are the pins available here (parity with the original binaries: unpinned)."""
import json
import math
import os

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from oracle import oracle as O
from squirrel_motion_planner_amd import scenes

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def orc(model_path):
    return O.Oracle(O.OracleRobot(model_path))


@pytest.fixture(scope="module")
def chain(model_path):
    with open(model_path) as f:
        return json.load(f)["chain"]


def np_fk(chain, q):
    """Independent chain FK: Rodrigues joint rotations, KDL segment pose joint(q) * f_tip (a fixed joint's pose is
    the identity, kdl_parser Joint(name, Joint::None))."""
    R, p = np.eye(3), np.zeros(3)
    for s in chain:
        ax = np.array(s["axis"], float)
        Rj, pj = np.eye(3), np.array(s["origin"], float) if s["type"] != "None" else np.zeros(3)
        if s["type"] == "RotAxis":
            Rj = Rotation.from_rotvec(ax * q[s["joint"]]).as_matrix()
        elif s["type"] == "TransAxis":
            pj = pj + ax * q[s["joint"]]
        Rf = np.array(s["ftip_R"], float).reshape(3, 3)
        pf = np.array(s["ftip_p"], float)
        Rs, ps = Rj @ Rf, Rj @ pf + pj
        R, p = R @ Rs, R @ ps + p
    return R, p


def random_configs(orobot, n, seed, base=1.5):
    rng = np.random.default_rng(seed)
    lo, hi = orobot.q_min.copy(), orobot.q_max.copy()
    lo[:2], hi[:2] = -base, base
    return rng.uniform(lo, hi, (n, 8))


def test_goal_quaternion_is_xyz_euler(orc):
    rng = np.random.default_rng(3)
    for _ in range(50):
        ee = np.concatenate([rng.uniform(-2, 2, 3), rng.uniform(-math.pi, math.pi, 3)])
        g = O.ik_goal(ee)
        ref = Rotation.from_euler("xyz", ee[3:]).as_quat()  # getFullPoseFromEEPose, birrt_star.cpp:1630-1645
        assert np.allclose(g[:3], ee[:3], rtol=0, atol=0)
        assert min(np.abs(g[3:] - ref).max(), np.abs(g[3:] + ref).max()) < 1e-12


def test_fk_pose_matches_numpy(orc, orobot, chain):
    Q = random_configs(orobot, 200, 1)
    ee, _ = orc.ik_fk_jac(Q)
    for q, e in zip(Q, ee):
        R, p = np_fk(chain, q)
        assert np.abs(e[:3] - p).max() < 1e-12
        ref = Rotation.from_matrix(R).as_quat()
        assert min(np.abs(e[3:] - ref).max(), np.abs(e[3:] + ref).max()) < 1e-9
        assert abs(np.linalg.norm(e[3:]) - 1) < 1e-12


def test_jacobian_matches_finite_differences(orc, orobot, chain):
    Q = random_configs(orobot, 40, 2)
    _, J = orc.ik_fk_jac(Q)
    h = 1e-6
    for q, Jq in zip(Q, J):
        # getJacobian casts to float (control_laws.cpp:5284-5293)
        assert np.array_equal(Jq, Jq.astype(np.float32).astype(np.float64))
        for c in range(8):
            qp, qm = q.copy(), q.copy()
            qp[c] += h
            qm[c] -= h
            Rp, pp = np_fk(chain, qp)
            Rm, pm = np_fk(chain, qm)
            dp = (pp - pm) / (2 * h)
            w = Rotation.from_matrix(Rp @ Rm.T).as_rotvec() / (2 * h)
            assert np.abs(Jq[:3, c] - dp).max() < 2e-6, (c, Jq[:3, c], dp)
            assert np.abs(Jq[3:, c] - w).max() < 2e-6, (c, Jq[3:, c], w)


def test_reached_poses_meet_the_deviation_band(orc, orobot, chain):
    """A REACHED run ends with every task coordinate inside its band (update_error_vec, control_laws.cpp:2222-2239),
    i.e. the hand within 5 mm of the goal and its orientation within the +-0.025 quaternion-vector band."""
    Q = random_configs(orobot, 60, 4)
    ee, _ = orc.ik_fk_jac(Q)
    rpy = Rotation.from_quat(ee[:, 3:]).as_euler("xyz")
    goals = np.column_stack([ee[:, :3], rpy])
    rng = np.random.default_rng(5)
    q0 = np.clip(Q + rng.normal(0, 0.3, Q.shape), orobot.q_min, orobot.q_max)
    r = orc.ik_solve(O.ik_tasks(goals, q0))
    assert r["reached"].sum() >= 25  # a local controller: some starts stall at joint limits (ADVANCED)
    for i in np.nonzero(r["reached"])[0]:
        q = r["q"][i]
        R, p = np_fk(chain, q)
        assert np.abs(goals[i, :3] - p).max() <= 0.005 + 1e-12
        ang = np.linalg.norm((Rotation.from_euler("xyz", goals[i, 3:]) * Rotation.from_matrix(R).inv()).as_rotvec())
        assert ang < 0.1
        inside = (q >= orobot.q_min) & (q <= orobot.q_max)
        assert np.all(inside | (q == q0[i]))  # a joint only moves inside its (float) limits (control_laws.cpp:3515)
        assert np.all(r["err"][i] == 0.0)
    for i in np.nonzero(r["reached"] == 0)[0]:
        assert r["iters"][i] == 1000


def test_goal_candidates_follow_the_reference_order():
    """findGoalPose tries start, +d, -d, +2d, -2d, ... while |diff| < pi (squirrel_8dof_planner.cpp:1172-1194)."""
    ee = [0.8, 0.3, 0.5, 1.57, 0.0, 0.3]
    cur = [0.1, -0.2, 0, 0, 0, 0, 0, 0]
    for disc, n in ((20.0, 17), (45.0, 7), (1.0, 361), (0.2, 361), (90.0, 3), (180.0, 1)):
        t, down = O.goal_candidates(ee, cur, disc)
        assert len(t) == n, (disc, len(t))  # the accumulated steps decide the last one (1 deg: 180 steps < pi)
        d = max(disc, 1.0) * (math.pi / 180.0)
        diffs, diff = [], 0.0
        while abs(diff) < math.pi:
            diffs.append(diff)
            diff *= -1
            diff += 0.0
            if diff >= 0.0:
                diff += d
        assert len(diffs) == n
        start = math.atan2(ee[1] - cur[1], ee[0] - cur[0])
        ang = t[:, 21] - 0.99
        assert np.allclose(ang, start + np.array(diffs), atol=1e-12)
        dist = 0.44 if down else 0.47
        assert np.allclose(np.hypot(ee[0] - t[:, 19], ee[1] - t[:, 20]), dist, atol=1e-12)
        arm = [-0.8, 0.8, 0.0, -1.5, 0.0] if down else [-1.2, 1.1, 0.0, 0.7, -1.5]
        assert np.array_equal(t[:, 22:27], np.tile(arm, (n, 1)))
        assert np.array_equal(t[:, 7:13], np.tile(O.IK_DEV[:, 0], (n, 1)))
    # downward: the hand's y axis (tf setRPY) within ~26 degrees of vertical (squirrel_8dof_planner.cpp:1140)
    assert O.goal_candidates([1, 1, 0.2, 1.57, 0, 0], cur, 20)[1]
    assert not O.goal_candidates([1, 1, 0.2, 0, 0, 0], cur, 20)[1]


def test_oracle_reproduces_golden_runs(orc):
    g = np.load(os.path.join(GOLD, "ik_golden.npz"))
    r = orc.ik_solve(O.ik_tasks(g["ee"], g["q_init"]))
    for k in ("q", "err", "manip"):
        assert np.array_equal(r[k], g[k], equal_nan=True), k
    for k in ("reached", "iters", "fallback"):
        assert np.array_equal(r[k], g[k]), k
    assert g["fallback"].max() > 0 and g["reached"].sum() > 20 and (g["reached"] == 0).sum() > 10


def test_find_goal_pose_semantics(orc, orobot, model_path):
    """First candidate (in the reference's order) whose run REACHED and whose pose is valid; 1 if poses were reached
    but all collide, 2 if none was reached."""
    sc = scenes.box_room()
    osc = O.OracleScene(sc.keys, sc.res)
    o = O.Oracle(O.OracleRobot(model_path), osc)
    cur = np.array(sc.start, float)
    for ee, disc in (([sc.start[0] + 0.6, sc.start[1] + 0.2, 0.5, 1.57, 0.0, 0.3], 20.0),
                     ([sc.start[0] - 0.5, sc.start[1] + 0.4, 0.3, 0.0, 1.57, 0.0], 30.0),
                     ([sc.start[0] + 0.3, sc.start[1] - 0.2, 2.5, 0.0, 0.0, 0.0], 45.0)):
        res, pose, tried, chosen, _ = o.find_goal_pose(ee, cur, disc, True, True)
        t, _ = O.goal_candidates(ee, cur, disc)
        r = o.ik_solve(t)
        v = o.check_configs(r["q"], True, True)
        ok = np.nonzero((r["reached"] == 1) & (v == 1))[0]
        if len(ok):
            assert res == 0 and chosen == ok[0] and tried == ok[0] + 1
            assert np.array_equal(pose, r["q"][ok[0]], equal_nan=True)
        else:
            assert res == (1 if r["reached"].any() else 2) and chosen == -1 and tried == len(t)
    assert res == 2  # the last goal is out of reach


def test_goal_straight_above_the_robot_propagates_nan(orc):
    """The reference's start angle is acos(0 / 0) when the goal is straight above the robot
    (squirrel_8dof_planner.cpp:1167-1169): every candidate base pose is NaN; the restatement keeps that."""
    t, _ = O.goal_candidates([0.5, 0.5, 1.0, 0.0, 0.0, 0.0], [0.5, 0.5, 0, 0, 0, 0, 0, 0], 45.0)
    assert np.isnan(t[:, 19:22]).all() and not np.isnan(t[:, 22:27]).any()
