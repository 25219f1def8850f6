"""CPU tests of the oracle (test infrastructure): known answers, internal consistency, golden regression."""
import math
import os

import numpy as np
import pytest

from oracle import octomap_bt, oracle as O
from squirrel_motion_planner_amd import scenes
from conftest import REF_CONFIG, have_reference

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32 10 rounds
    assert O.philox([0, 0, 0, 0], [0, 0]).tolist() == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert O.philox([0xffffffff] * 4, [0xffffffff] * 2).tolist() == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert O.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]).tolist() == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_u01_range_and_mean():
    rng = np.random.default_rng(0)
    ctr = rng.integers(0, 2**32, (20000, 4), dtype=np.uint64).astype(np.uint32)
    u = O.u01(12345, 7, ctr)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.01
    assert np.array_equal(u, O.u01(12345, 7, ctr))


def test_portable_sincos_accuracy():
    x = np.concatenate([np.linspace(-10, 10, 20001), np.array([0.0, -0.0, math.pi, -math.pi, 1e-300, 123.456])])
    s, c = O.sincos(x)
    ref_s = np.sin(x)
    ref_c = np.cos(x)
    ulp = np.spacing(np.maximum(np.abs(ref_s), 1e-300))
    assert np.all(np.abs(s - ref_s) <= 4 * np.maximum(ulp, 1e-16))
    assert np.all(np.abs(c - ref_c) <= 4 * np.maximum(np.spacing(np.abs(ref_c)), 1e-16))


def test_body_fk_matches_tree_recursion(orobot, model_path):
    """Rigid-body collapse vs the faithful per-link KDL tree recursion: same geometry."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    model = json.load(open(model_path))
    orc = O.Oracle(orobot)
    rng = np.random.default_rng(1)
    q = np.column_stack([rng.uniform(-3, 3, 50), rng.uniform(-3, 3, 50)] +
                        [rng.uniform(orobot.q_min[j], orobot.q_max[j], 50) for j in range(2, 8)])
    frames, _ = orc.fk(q)                    # faithful tree (n, 39, 12)
    bodies = orc.body_fk(q)                  # collapsed (n, 6, 12)
    for b, li in enumerate(model["bodies"]):
        assert np.array_equal(bodies[:, b], frames[:, li])  # body frames are the tree recursion itself
    # sphere centres: body pre-composition vs per-link frames
    for s in model["spheres"]:
        Tl = frames[:, s["link"]]
        cw = np.einsum("nij,j->ni", Tl[:, :9].reshape(-1, 3, 3), s["c"]) + Tl[:, 9:]
        Tb = bodies[:, s["body"]]
        cb = np.einsum("nij,j->ni", Tb[:, :9].reshape(-1, 3, 3), s["cb"]) + Tb[:, 9:]
        assert np.max(np.abs(cw - cb)) < 1e-12


def test_folding_poses_valid_and_random_mix(orobot):
    sc = scenes.empty_room()
    orc = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res))
    assert orc.check_configs([sc.start, sc.goal]).tolist() == [1, 1]
    rng = np.random.default_rng(2)
    q = np.column_stack([rng.uniform(-2, 2, 3000), rng.uniform(-2, 2, 3000)] +
                        [rng.uniform(orobot.q_min[j], orobot.q_max[j], 3000) for j in range(2, 8)])
    v = orc.check_configs(q)
    assert 0.2 < v.mean() < 0.9  # both outcomes well represented
    # self / map switches (isInCollision(q, self, map), collision_checker.hpp:104-121)
    assert np.all(orc.check_configs(q, False, False) == 1)
    vs = orc.check_configs(q, True, False)
    vm = orc.check_configs(q, False, True)
    assert np.array_equal(v, vs & vm)


def test_octomap_bt_roundtrip():
    rng = np.random.default_rng(3)
    keys = np.unique(rng.integers(32768 - 40, 32768 + 40, (500, 3)), axis=0)
    res, k2 = octomap_bt.read_bt(octomap_bt.write_bt(keys, 0.05))
    assert res == 0.05
    assert np.array_equal(np.unique(k2, axis=0), keys)


@pytest.mark.parametrize("room", ["room3", "room4", "room5"])
def test_room_fixture(room):
    f = np.load(os.path.join(GOLD, room + "_keys.npz"))
    assert float(f["res"]) == 0.05
    assert len(f["keys"]) in (5548, 4192, 4408)
    if have_reference():
        res, keys = octomap_bt.read_bt(open(os.path.join(REF_CONFIG, room + ".bt"), "rb").read())
        assert np.array_equal(np.unique(keys, axis=0), np.unique(f["keys"].astype(np.int64), axis=0))


def test_oracle_scene_box_gap_matches_bruteforce():
    """d2 = squared box-to-box gap (voxels) to the nearest occupied cell: sum over axes of max(|du| - 1, 0)^2."""
    rng = np.random.default_rng(4)
    keys = 32768 + rng.integers(0, 12, (30, 3))
    g = O.OracleScene(keys, 0.05)
    occ = g.occ
    pts = np.argwhere(occ)
    idx = np.argwhere(np.ones_like(occ))
    gap = np.maximum(np.abs(idx[:, None, :] - pts[None, :, :]) - 1, 0)
    d2 = (gap ** 2).sum(-1).min(1)
    assert np.array_equal(g.d2, np.minimum(d2, 65535).astype(np.uint16))


def test_box_gap_is_a_lower_bound_of_the_exact_map_test():
    """Random spheres: whenever the prefilter says free (d2 > floor(((r + 1e-6)/res)^2)), no occupied box is
    within r of the centre (brute force over every occupied box)."""
    rng = np.random.default_rng(5)
    keys = 32768 + rng.integers(0, 16, (60, 3))
    g = O.OracleScene(keys, 0.05)
    occ_idx = np.argwhere(g.occ)  # (k, j, i)
    lo = np.stack([g.ox + occ_idx[:, 2] * g.res, g.oy + occ_idx[:, 1] * g.res, g.oz + occ_idx[:, 0] * g.res], 1)
    hi = lo + g.res
    d2 = g.d2.reshape(g.occ.shape)
    n_free = 0
    for _ in range(3000):
        c = np.array([g.ox, g.oy, g.oz]) + rng.uniform(0, 1, 3) * np.array([g.nx, g.ny, g.nz]) * g.res
        r = rng.uniform(0.001, 0.3)
        ci = np.floor((c - np.array([g.ox, g.oy, g.oz])) / g.res).astype(int)
        T = np.floor(((r + 1e-6) / g.res) ** 2)
        if d2[ci[2], ci[1], ci[0]] > T:
            n_free += 1
            gap = np.maximum(np.maximum(lo - c, c - hi), 0.0)
            assert (gap ** 2).sum(1).min() > r * r
    assert n_free > 500


@pytest.mark.parametrize("name", ["c1_direct", "c2_boxes_300", "c2_boxes_yaml", "c4_passage"])
def test_oracle_golden_regression(name):
    """The oracle reproduces its committed seeded runs bit for bit (pins the restatement)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(GOLD, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    _, r = mg.plan_case(name)
    g = np.load(os.path.join(GOLD, "plan_%s.npz" % name))
    assert r["status"] == int(g["status"])
    assert r["iterations"] == int(g["iterations"]) and r["first_iter"] == int(g["first_iter"])
    assert r["checked"] == int(g["checked"]) and r["valid"] == int(g["valid"])
    for k in ("start_parent", "goal_parent"):
        assert np.array_equal(r[k], g[k])
    for k in ("start_cost", "goal_cost", "start_conf", "goal_conf", "path"):
        assert np.array_equal(r[k], g[k]), k
    assert np.array_equal(np.array(r["cost"]), g["cost"])


def test_oracle_invalid_start_goal(orobot):
    sc = scenes.box_room()
    orc = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res))
    inside_wall = [5.05, 0.0, 0.0] + scenes.ARM_FOLDED
    assert orc.plan(inside_wall, sc.goal, env_x=sc.env_x, env_y=sc.env_y)["status"] == -2
    assert orc.plan(sc.start, inside_wall, env_x=sc.env_x, env_y=sc.env_y)["status"] == -3


def test_oracle_tree_invariants(orobot):
    """no_two_parents_check / cost consistency (birrt_star.cpp:6812-6860) on a seeded run."""
    sc = scenes.box_room()
    orc = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res))
    r = orc.plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=250, seed=11)
    for t in ("start", "goal"):
        par = r[t + "_parent"]
        assert par[0] == 0
        assert np.all(par[1:] < np.arange(1, len(par)) + 10**9)
        # every node reaches the root (no loops)
        for i in range(len(par)):
            j, steps = i, 0
            while j != 0:
                j = par[j]
                steps += 1
                assert steps <= len(par)
    if r["status"] == 0:
        p = r["path"]
        assert np.array_equal(p[0], np.array(sc.start))


def test_collision_listing_agrees_with_validity():
    """orc_collisions (getCollisions, CC:123-132, 594-630) lists something exactly when isInCollision is true (no
    disabled links), self pairs in model pair order, map links sorted by name."""
    model = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "squirrel_motion_planner_amd",
                         "data", "robotino_model.json")
    sc = scenes.box_room()
    orc = O.Oracle(O.OracleRobot(model), O.OracleScene(sc.keys, sc.res))
    rng = np.random.default_rng(3)
    n = 300
    q = np.column_stack([rng.uniform(-5, 5, n), rng.uniform(-5, 5, n), rng.uniform(-math.pi, math.pi, n)] +
                        [rng.uniform(lo, hi, n) for lo, hi in zip([-1.2, -1.7, -1.8, -2.4, -2.9], [1.5, 2.6, 1.8, 2.4, 2.9])])
    valid = orc.check_configs(q)
    pair_order = {(a, b): k for k, (a, b) in enumerate(
        (orc.robot.model["links"][a]["name"], orc.robot.model["links"][b]["name"])
        for a, b in zip(orc.robot.pair_a, orc.robot.pair_b))}
    listed = 0
    for qi, v in zip(q, valid):
        s, m = orc.collisions(qi)
        assert (not s and not m) == bool(v)
        assert m == sorted(m) and [pair_order[p] for p in s] == sorted(pair_order[p] for p in s)
        listed += bool(s) + bool(m)
    assert listed > 50


def test_openmp_scans_plan_the_same_trees(orobot):
    """The all-core CPU baseline (OpenMP scans as BS:4092 / BS:4283) plans exactly what the sequential oracle plans."""
    sc = scenes.box_room()
    orc = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res))
    kw = dict(env_x=sc.env_x, env_y=sc.env_y, seed=5, max_iter=400, opt_thresh=-math.inf)
    a = orc.plan(sc.start, sc.goal, threads=1, **kw)
    b = orc.plan(sc.start, sc.goal, threads=4, **kw)
    for k in ("iterations", "checked", "valid", "n_start", "n_goal", "conn_a", "conn_b"):
        assert a[k] == b[k], k
    assert a["cost"] == b["cost"]
    assert np.array_equal(a["start_parent"], b["start_parent"]) and np.array_equal(a["goal_conf"], b["goal_conf"])
    assert np.array_equal(a["path"], b["path"])


def test_oracle_resume_equals_one_run(orobot):
    """orc_resume_*: the oracle continued from its own state after 700 iterations plans exactly the run of 1500
    iterations (trees, counters, costs, path) -- the mechanism the large-tree parity and timing use on GPU states."""
    import math
    from squirrel_motion_planner_amd import scenes
    sc = scenes.box_room()
    kw = dict(env_x=sc.env_x, env_y=sc.env_y, seed=1, opt_thresh=-math.inf)
    o1 = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res))
    st = o1.export_state(o1.plan(sc.start, sc.goal, max_iter=700, **kw))
    r2 = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res)).resume(sc.start, sc.goal, st, max_iter=1500, **kw)
    r3 = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res)).plan(sc.start, sc.goal, max_iter=1500, **kw)
    for k in ("iterations", "checked", "valid", "first_iter", "last_iter", "n_start", "n_goal", "edges_start",
              "edges_goal", "rewires_start", "rewires_goal", "conn_b", "conn_a", "conn_start", "status"):
        assert r2[k] == r3[k], k
    assert r2["cost"] == r3["cost"]
    for n in ("start", "goal"):
        for f in ("parent", "conf", "cost"):
            assert np.array_equal(r2[n + "_" + f], r3[n + "_" + f])
    assert np.array_equal(r2["path"], r3["path"])
