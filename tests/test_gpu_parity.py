"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on the same seeded inputs.

Bar: bit-exact for integers (tree parent ids, connection order, counters) and -- by construction of the
shared fp64 arithmetic -- bit-exact for configurations, costs and waypoints too (the north-star tolerance
for joint waypoints is 1e-6; the tests assert equality and report the max deviation on failure).
"""
import ctypes
import math
import os

import numpy as np
import pytest

from oracle import octomap_bt, oracle as O
from squirrel_motion_planner_amd import _lib as L
from squirrel_motion_planner_amd import scenes
from squirrel_motion_planner_amd.planner import BiRRTstarPlanner, GpuPlanner, Robot, Scene

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
_pd = ctypes.POINTER(ctypes.c_double)


@pytest.fixture(scope="module")
def robot():
    return Robot()


@pytest.fixture(scope="module")
def gp(robot):
    return GpuPlanner(robot)


_SCENES = {}


def scene_pair(name):
    if name not in _SCENES:
        if name.startswith("room"):
            f = np.load(os.path.join(GOLD, name + "_keys.npz"))
            keys = np.concatenate([f["keys"].astype(np.int64), scenes.floor_keys([0.0, 0.0], 0.05, 3.0)])
            sc = scenes.Scene(name, keys, 0.05, [0, 0, 0] + scenes.ARM_FOLDED, [1, 1, 0] + scenes.ARM_UNFOLDED,
                              (0, 0), (0, 0))
            sc.env_x, sc.env_y = sc.bounds()
        else:
            sc = {"c1": scenes.empty_room, "c2": scenes.box_room, "c4": scenes.narrow_passage,
                  "c5": scenes.clutter_cloud}[name]()
        _SCENES[name] = (sc, Scene.from_keys(sc.keys, sc.res), O.OracleScene(sc.keys, sc.res))
    return _SCENES[name]


def random_configs(sc, n, seed, orobot):
    rng = np.random.default_rng(seed)
    (x0, x1), (y0, y1) = sc.env_x, sc.env_y
    return np.column_stack([rng.uniform(x0, x1, n), rng.uniform(y0, y1, n)] +
                           [rng.uniform(orobot.q_min[j] - 0.3, orobot.q_max[j] + 0.3, n) for j in range(2, 8)])


# ------------------------------------------------------------------------------------------ arithmetic
def test_sincos_bitwise():
    x = np.concatenate([np.linspace(-20, 20, 100001), np.random.default_rng(0).uniform(-1e3, 1e3, 10000)])
    s, c = np.zeros_like(x), np.zeros_like(x)
    L.check(L.lib().smp_probe_sincos(0, x.ctypes.data_as(_pd), len(x), s.ctypes.data_as(_pd), c.ctypes.data_as(_pd)))
    os_, oc = O.sincos(x)
    assert np.array_equal(s, os_) and np.array_equal(c, oc)


def test_philox_u01_bitwise():
    rng = np.random.default_rng(1)
    ctr = rng.integers(0, 2**32, (50000, 4), dtype=np.uint64).astype(np.uint32)
    out = np.zeros(len(ctr))
    L.check(L.lib().smp_probe_u01(0, 0x123456789ABCDEF, 17, ctr.ctypes.data_as(ctypes.c_void_p), len(ctr),
                                  out.ctypes.data_as(_pd)))
    assert np.array_equal(out, O.u01(0x123456789ABCDEF, 17, ctr))


def test_sqrt_div_correctly_rounded():
    rng = np.random.default_rng(2)
    a = np.concatenate([rng.uniform(0, 100, 200000), rng.uniform(0, 1e-8, 1000), np.array([0.0, 1.0, 2.0, 4.0])])
    b = np.concatenate([rng.uniform(0.1, 50, len(a) - 4), np.array([3.0, 7.0, 20.0, 0.5])])
    sq, dv = np.zeros_like(a), np.zeros_like(a)
    L.check(L.lib().smp_probe_sqrt_div(0, a.ctypes.data_as(_pd), b.ctypes.data_as(_pd), len(a),
                                       sq.ctypes.data_as(_pd), dv.ctypes.data_as(_pd)))
    assert np.array_equal(sq, np.sqrt(a))
    assert np.array_equal(dv, a / b)


def test_fk_bitwise(gp, orobot):
    sc, _, osc = scene_pair("c2")
    q = random_configs(sc, 4000, 3, orobot)
    nb = len(orobot.model["bodies"])
    fr = np.zeros((len(q), nb, 12))
    z = np.zeros(len(q))
    qq = np.ascontiguousarray(q)
    L.check(L.lib().smp_probe_fk(gp.h, qq.ctypes.data_as(_pd), len(q), fr.ctypes.data_as(_pd), z.ctypes.data_as(_pd)))
    orc = O.Oracle(orobot, osc)
    assert np.array_equal(fr, orc.body_fk(q))
    _, oz = orc.fk(q)
    assert np.array_equal(z, oz)


# ------------------------------------------------------------------------------------------ collision
@pytest.mark.parametrize("name", ["c1", "c2", "c4", "room3"])
@pytest.mark.parametrize("flags", [(1, 1), (1, 0), (0, 1)])
def test_check_configs_parity(gp, orobot, name, flags):
    sc, gscene, osc = scene_pair(name)
    gp.set_scene(gscene)
    gp.set_disabled_map_links([])
    q = random_configs(sc, 100000, hash(name) % 1000, orobot)
    v = gp.check_configs(q, *flags)
    ov = O.Oracle(orobot, osc).check_configs(q, *flags)
    assert v.dtype == np.uint8
    mism = np.flatnonzero(v != ov)
    assert len(mism) == 0, "mismatches at %s" % mism[:10]
    assert 0.05 < v.mean() < 0.99


@pytest.mark.parametrize("name", ["c2", "room3", "c5"])
@pytest.mark.parametrize("tile", [-1, -2, -4, -8, 8])
def test_job_tile_shapes_parity(gp, orobot, name, tile):
    """The helpers' job tiles (collide_wide: ct = -tile configurations spread over the workgroup's 8 wavefronts, the map
    and self tests split among them) decide every configuration as the oracle does, with self / map on and off.  The
    configurations include points along tree-like edges near obstacles (many candidate spheres per configuration)."""
    sc, gscene, osc = scene_pair(name)
    gp.set_scene(gscene)
    gp.set_disabled_map_links([])
    rng = np.random.default_rng(5)
    q = random_configs(sc, 20000, 11, orobot)
    a, b = q[rng.integers(0, len(q), 500)], q[rng.integers(0, len(q), 500)]
    t = np.linspace(0.0, 1.0, 21)[None, :, None]
    q = np.concatenate([q, (a[:, None, :] + t * (b - a)[:, None, :]).reshape(-1, 8)])
    soa = np.ascontiguousarray(q.T)
    orc = O.Oracle(orobot, osc)
    for flags in [(1, 1), (1, 0), (0, 1)]:
        v = np.zeros(len(q), np.uint8)
        L.check(L.lib().smp_probe_check_shape(gp.h, soa.ctypes.data_as(_pd), len(q), flags[0], flags[1], tile, 2048,
                                              v.ctypes.data_as(ctypes.c_void_p)))
        ov = orc.check_configs(q, *flags)
        mism = np.flatnonzero(v != ov)
        assert len(mism) == 0, "tile %d flags %s: mismatches at %s" % (tile, flags, mism[:10])
        assert 0.01 < v.mean() < 0.99  # both outcomes exercised (the 2 cm clutter leaves ~4 % of them free)


def test_disabled_map_links(gp, orobot):
    sc, gscene, osc = scene_pair("c2")
    gp.set_scene(gscene)
    links = ["base_body_link", "shell_base_link_front", "hand_wrist_link"]
    gp.set_disabled_map_links(links)
    me = np.array([0 if n in links else 1 for n in orobot.link_names], np.uint8)
    q = random_configs(sc, 50000, 9, orobot)
    v = gp.check_configs(q)
    ov = O.Oracle(orobot, osc, map_enabled=me).check_configs(q)
    gp.set_disabled_map_links([])
    assert np.array_equal(v, ov)


def test_check_empty_and_single(gp):
    assert len(gp.check_configs(np.zeros((0, 8)))) == 0
    sc, gscene, _ = scene_pair("c1")
    gp.set_scene(gscene)
    assert gp.check_configs([sc.start]).tolist() == [1]


# ------------------------------------------------------------------------------------------ planner
def run_both(gp, orobot, name, seed, iters, **pk):
    sc, gscene, osc = scene_pair(name)
    gp.set_scene(gscene)
    gp.set_disabled_map_links([])
    q = GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=iters, seed=seed)
    r = gp.plan(q)
    okw = dict(max_iter=iters, seed=seed)
    if "near_threshold" in pk:
        okw["near_r"] = pk["near_threshold"]
    if "step_factor" in pk:
        okw["step"] = pk["step_factor"]
    o = O.Oracle(orobot, osc).plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, **okw)
    return sc, r, o


def assert_same_run(gp, r, o):
    assert r["status"] == {0: 0, 1: L.SMP_ERR_NO_SOLUTION}[o["status"]]
    assert r["iterations"] == o["iterations"]
    assert r["first_solution_iter"] == o["first_iter"]
    assert r["configs_checked"] == o["checked"]
    assert r["configs_valid"] == o["valid"]
    assert r["nodes_start"] == o["n_start"] and r["nodes_goal"] == o["n_goal"]
    assert r["rewires_start"] == o["rewires_start"] and r["rewires_goal"] == o["rewires_goal"]
    assert r["edges_start"] == o["edges_start"] and r["edges_goal"] == o["edges_goal"]
    for w, name in ((0, "start"), (1, "goal")):
        par, conf, cost = gp.tree(w)
        assert np.array_equal(par, o[name + "_parent"]), name
        assert np.array_equal(conf, o[name + "_conf"]), (name, np.abs(conf - o[name + "_conf"]).max())
        assert np.array_equal(cost, o[name + "_cost"]), name
    assert r["cost_best"] == o["cost"]
    if r["status"] == 0:
        assert r["connected_tree_is_start"] == o["conn_start"]
        assert r["conn_node_b"] == o["conn_b"] and r["conn_node_a"] == o["conn_a"]
        assert r["path"].shape == o["path"].shape
        assert np.max(np.abs(r["path"] - o["path"])) <= 1e-6
        assert np.array_equal(r["path"], o["path"])
    assert np.array_equal(r["cost_rows"][:, [0, 2, 3, 4]], o["cost_rows"][:, [0, 2, 3, 4]])


@pytest.mark.parametrize("name,seed,iters", [("c1", 1, 50), ("c2", 3, 300), ("c2", 8, 600), ("c4", 2, 400),
                                             ("room3", 4, 300)])
def test_planner_parity(gp, orobot, name, seed, iters):
    sc, r, o = run_both(gp, orobot, name, seed, iters)
    assert_same_run(gp, r, o)


@pytest.mark.parametrize("name,seed,samples", [("c2", 11, 30000), ("c4", 2, 20000), ("room3", 2, 20000)])
def test_planner_parity_sample_budget(orobot, robot, name, seed, samples):
    """The bench's budget: collision-checked configurations, path_optimality_threshold = -inf."""
    gp2 = GpuPlanner(robot, path_optimality_threshold=-np.inf)
    sc, gscene, osc = scene_pair(name)
    gp2.set_scene(gscene)
    r = gp2.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, samples=samples, seed=seed))
    o = O.Oracle(orobot, osc).plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_checked=samples,
                                   seed=seed, opt_thresh=-np.inf)
    if o["iterations"] > 0:  # (room3 connects directly before the loop, birrt_star.cpp:1072-1075)
        assert o["checked"] >= samples
    assert_same_run(gp2, r, o)


@pytest.mark.parametrize("seed", [1, 1001, 2001])
def test_planner_parity_bench_workload(orobot, robot, seed):
    """bench.py's C2 step at full size (default steps 0-2: seeds 1, 1001, 2001; 1e6 collision-checked samples,
    path_optimality_threshold = -inf, default helpers and scouts): both trees, costs and path bit for bit."""
    gp2 = GpuPlanner(robot, path_optimality_threshold=-np.inf)
    sc, gscene, osc = scene_pair("c2")
    gp2.set_scene(gscene)
    r = gp2.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, samples=1_000_000, seed=seed))
    o = O.Oracle(orobot, osc).plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_checked=1_000_000,
                                   seed=seed, opt_thresh=-np.inf)
    assert o["checked"] >= 1_000_000 and r["status"] == 0
    assert r["scout"] >= 1 and r["helpers"] > 0  # the run-ahead path the bench measures
    assert_same_run(gp2, r, o)


@pytest.mark.parametrize("helpers", [-1, 1, 7])
def test_planner_parity_helper_counts(orobot, robot, helpers):
    """The query alone on its workgroup (-1) and with helper workgroups sharing its collision tiles."""
    gp2 = GpuPlanner(robot, helpers=helpers)
    sc, r, o = run_both(gp2, orobot, "c2", 8, 400)
    assert_same_run(gp2, r, o)


@pytest.mark.parametrize("scouts", [2, 3, 4, 6, 8])
def test_planner_parity_scout_counts(orobot, robot, scouts):
    """Two, three and four scouts taking the iterations in turn before the first solution (records up to
    four iterations ahead, patched by the leader), across the first solution and 2000 iterations after it."""
    gp2 = GpuPlanner(robot, helpers=63, scout=scouts, path_optimality_threshold=-np.inf)
    sc, gscene, osc = scene_pair("c2")
    gp2.set_scene(gscene)
    r = gp2.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=2000, seed=5))
    o = O.Oracle(orobot, osc).plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=2000, seed=5,
                                   opt_thresh=-np.inf)
    assert r["scout"] == scouts
    assert_same_run(gp2, r, o)


@pytest.mark.parametrize("n_pts", [10, 21, 22, 32])
def test_planner_parity_segment_counts(orobot, robot, n_pts):
    """num_traj_segments_interp other than the default 20, across the first solution: 21 is the largest count whose
    via-chain segment norms take one lane each per norm (via_chain_w's lane groups of 21), 22 and up take the
    three-norms-per-lane path, 32 = MAX_PTS; the scouts' records, the helpers' tiles and the edge costs all change."""
    gp2 = GpuPlanner(robot, num_traj_segments=n_pts, path_optimality_threshold=-np.inf)
    sc, gscene, osc = scene_pair("c2")
    gp2.set_scene(gscene)
    r = gp2.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=1500, seed=7))
    o = O.Oracle(orobot, osc).plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=1500, seed=7,
                                   opt_thresh=-np.inf, n_pts=n_pts)
    assert r["status"] == 0 and r["scout"] >= 1
    assert_same_run(gp2, r, o)


def test_planner_parity_yaml_profile(orobot, robot):
    gp2 = GpuPlanner(robot, near_threshold=1.5, step_factor=0.6)
    sc, r, o = run_both(gp2, orobot, "c2", 5, 200, near_threshold=1.5, step_factor=0.6)
    assert_same_run(gp2, r, o)


@pytest.mark.parametrize("name", ["c1", "c2", "c4"])
def test_golden_fixture(gp, name):
    """GPU run reproduces the committed oracle fixture (no oracle needed at run time)."""
    case = {"c1": "c1_direct", "c2": "c2_boxes_300", "c4": "c4_passage"}[name]
    g = np.load(os.path.join(GOLD, "plan_%s.npz" % case))
    sc, gscene, _ = scene_pair(name)
    gp.set_scene(gscene)
    seeds = {"c1_direct": (1, 50), "c2_boxes_300": (3, 300), "c4_passage": (2, 400)}
    seed, iters = seeds[case]
    r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=iters, seed=seed))
    assert r["configs_checked"] == int(g["checked"])
    par, conf, cost = gp.tree(0)
    assert np.array_equal(par, g["start_parent"]) and np.array_equal(conf, g["start_conf"])
    assert np.array_equal(r["path"], g["path"])


def test_invalid_start_goal(gp):
    sc, gscene, _ = scene_pair("c2")
    gp.set_scene(gscene)
    wall = [5.05, 0.0, 0.0] + scenes.ARM_FOLDED
    r = gp.plan(GpuPlanner.make_query(wall, sc.goal, sc.env_x, sc.env_y, iterations=10))
    assert r["status"] == L.SMP_ERR_START_INVALID
    r = gp.plan(GpuPlanner.make_query(sc.start, wall, sc.env_x, sc.env_y, iterations=10))
    assert r["status"] == L.SMP_ERR_GOAL_INVALID


def test_no_solution_small_budget(gp, orobot):
    sc, r, o = run_both(gp, orobot, "c2", 3, 5)
    assert o["status"] == 1
    assert_same_run(gp, r, o)


def test_batch_equals_single(gp):
    sc, gscene, _ = scene_pair("c2")
    gp.set_scene(gscene)
    qs = [GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=150, seed=s, query_id=s)
          for s in range(4)]
    batch = gp.plan_batch(qs)
    for q, b in zip(qs, batch):
        s = gp.plan(q)
        assert b["status"] == s["status"] and b["configs_checked"] == s["configs_checked"]
        assert np.array_equal(b["path"], s["path"])


def test_batch_repeated_is_deterministic(gp):
    """Race detector: the 4-query batch (every CU busy: leaders, scouts, helpers) repeated 30 times gives the same
    runs each time.  Caught a stale sample taken from empty pre-solution records and a barrier desync after a
    record time-out, both timing-dependent."""
    sc, gscene, _ = scene_pair("c2")
    gp.set_scene(gscene)
    qs = [GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=150, seed=s, query_id=s)
          for s in range(4)]
    ref = [gp.plan(q)["configs_checked"] for q in qs]
    for _ in range(30):
        assert [r["configs_checked"] for r in gp.plan_batch(qs)] == ref


def _same_query_result(r, o):
    assert r["status"] == {0: 0, 1: L.SMP_ERR_NO_SOLUTION}[o["status"]]
    for k_r, k_o in (("iterations", "iterations"), ("first_solution_iter", "first_iter"), ("configs_checked", "checked"),
                     ("configs_valid", "valid"), ("nodes_start", "n_start"), ("nodes_goal", "n_goal"),
                     ("rewires_start", "rewires_start"), ("rewires_goal", "rewires_goal")):
        assert r[k_r] == o[k_o], k_r
    assert r["cost_best"] == o["cost"]
    if r["status"] == 0:
        assert np.array_equal(r["path"], o["path"])


def test_c3_random_queries_batch(orobot, robot):
    """C3: random (start, goal) pairs on the C2 scene (scenes.random_queries, seed 7), one batch of 8 queries sharing
    the chip (each with its own Philox stream, query_id k); every query equals its own oracle run."""
    gp2 = GpuPlanner(robot)
    sc, gscene, osc = scene_pair("c2")
    gp2.set_scene(gscene)
    pairs = scenes.random_queries(sc, 8, seed=7, check=lambda q: bool(gp2.check_configs([q])[0]))
    assert len(pairs) == 8
    qs = [GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, iterations=200, seed=7, query_id=k)
          for k, (s, g) in enumerate(pairs)]
    rs = gp2.plan_batch(qs)
    orc = O.Oracle(orobot, osc)
    for k, ((s, g), r) in enumerate(zip(pairs, rs)):
        o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_iter=200, seed=7, query=k)
        _same_query_result(r, o)


def test_c3_bench_share_full_budget(orobot, robot):
    """bench.py --workload c3 step 0 at full size: the 8 queries of one GPU's share (seed 1, query_id k), 1e6
    collision-checked samples each, path_optimality_threshold = -inf, queries sharing the chip's helpers."""
    gp2 = GpuPlanner(robot, path_optimality_threshold=-np.inf)
    sc, gscene, osc = scene_pair("c2")
    gp2.set_scene(gscene)
    pairs = scenes.random_queries(sc, 8, seed=7, check=lambda q: bool(gp2.check_configs([q])[0]))
    qs = [GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, samples=1_000_000, seed=1, query_id=k)
          for k, (s, g) in enumerate(pairs)]
    rs = gp2.plan_batch(qs)
    orc = O.Oracle(orobot, osc)
    for k, ((s, g), r) in enumerate(zip(pairs, rs)):
        o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_checked=1_000_000, seed=1, query=k,
                     opt_thresh=-np.inf)
        assert o["checked"] >= 1_000_000 or o["iterations"] == 0
        _same_query_result(r, o)


def test_many_queries_reprovisioned_match_oracle(orobot, robot):
    """Many queries with staggered budgets (24 random C3 pairs, 40 .. 730 iterations): launches end as quarters of
    the running queries finish and the finished queries' CUs go to the others (more helpers, scouts appearing), several
    times in one call (DESIGN.md "Many queries"); every query still equals its oracle run."""
    gp2 = GpuPlanner(robot)
    sc, gscene, osc = scene_pair("c2")
    gp2.set_scene(gscene)
    pairs = scenes.random_queries(sc, 24, seed=7, check=lambda q: bool(gp2.check_configs([q])[0]))
    assert len(pairs) == 24
    budgets = [40 + 30 * k for k in range(24)]
    qs = [GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, iterations=b, seed=5, query_id=k)
          for k, ((s, g), b) in enumerate(zip(pairs, budgets))]
    rs = gp2.plan_batch(qs)
    _, _, launches = gp2.last_kernel_ms()
    assert launches >= 4  # re-provisioned more than once
    orc = O.Oracle(orobot, osc)
    for k, ((s, g), r) in enumerate(zip(pairs, rs)):
        o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_iter=budgets[k], seed=5, query=k)
        _same_query_result(r, o)


def test_single_query_relaunched_equals_one_launch(orobot, robot, monkeypatch):
    """A single query runs its whole budget in one launch; forced into launches of 64 iterations (SMP_CHUNK0, the loop
    state resumed from QState each time, scouts and helpers restarted) it plans the identical trees, path and counters,
    and both equal the oracle."""
    gp2 = GpuPlanner(robot, path_optimality_threshold=-math.inf)
    sc, gscene, osc = scene_pair("c2")
    gp2.set_scene(gscene)
    q = GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=700, seed=3)
    one = gp2.plan(q)
    assert gp2.last_kernel_ms()[2] == 1
    t_one = [gp2.tree(w) for w in (0, 1)]
    monkeypatch.setenv("SMP_CHUNK0", "64")
    many = gp2.plan(q)
    assert gp2.last_kernel_ms()[2] >= 4
    for k in ("status", "iterations", "configs_checked", "configs_valid", "nodes_start", "nodes_goal",
              "first_solution_iter", "rewires_start", "rewires_goal"):
        assert one[k] == many[k], k
    assert np.array_equal(one["path"], many["path"]) and one["cost_best"] == many["cost_best"]
    for w in (0, 1):
        par, conf, cost = gp2.tree(w)
        assert np.array_equal(par, t_one[w][0]) and np.array_equal(conf, t_one[w][1])
        assert np.array_equal(cost, t_one[w][2])
    o = O.Oracle(orobot, osc).plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=700, seed=3,
                                   opt_thresh=-np.inf)
    _same_query_result(one, o)


@pytest.fixture(scope="module")
def c5_pair():
    sc = scenes.clutter_cloud()
    return sc, Scene.from_keys(sc.keys, sc.res), O.OracleScene(sc.keys, sc.res)


def test_c5_clutter_2cm_check_and_plan(orobot, robot, c5_pair):
    """C5: 2 cm dense clutter from the 2e6-point synthetic cloud (500 x 500 x 100 cells): per-configuration
    validity and a short planning run equal the oracle."""
    sc, gscene, osc = c5_pair
    gp2 = GpuPlanner(robot)
    gp2.set_scene(gscene)
    q = random_configs(sc, 20000, 5, orobot)
    v = gp2.check_configs(q)
    assert np.array_equal(v, O.Oracle(orobot, osc).check_configs(q, 1, 1))
    assert 0.02 < v.mean() < 0.99
    r = gp2.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=300, seed=1))
    o = O.Oracle(orobot, osc).plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=300, seed=1)
    assert_same_run(gp2, r, o)


@pytest.mark.parametrize("helpers,scout", [(2, 0), (29, 2)])
def test_c5_informed_samples_from_the_ring(orobot, robot, c5_pair, helpers, scout):
    """C5 query 0 (first solution at iteration 2136) to 3000 iterations with the run-ahead sampler serving the
    informed (post-solution) samples: helpers = 2 is one tile helper + the sampler, no scout.  A ring sample drawn with
    another cost bound than the leader's once slipped in here (trees equal to the oracle's up to the solution, then
    not); the leader now takes a slot only if its sampling parameters equal its own."""
    sc, gscene, osc = c5_pair
    gp2 = GpuPlanner(robot, path_optimality_threshold=-np.inf, helpers=helpers, scout=scout)
    gp2.set_scene(gscene)
    s, g = scenes.random_queries(sc, 1, seed=7, check=lambda q: bool(gp2.check_configs([q])[0]))[0]
    r = gp2.plan(GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, iterations=3000, seed=1, query_id=0))
    assert r["samples_precomputed"] > 2000  # the ring served most iterations, before and after the solution
    o = O.Oracle(orobot, osc).plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_iter=3000, seed=1, query=0,
                                   opt_thresh=-np.inf)
    assert o["first_iter"] < 2500
    assert_same_run(gp2, r, o)


def test_c5_bench_share_full_budget(orobot, robot, c5_pair):
    """bench.py --workload c5 step 0 at full size: 8 random queries on the 2 cm clutter scene (seed 7), 1e6
    collision-checked samples each, path_optimality_threshold = -inf; every query equals its oracle run."""
    sc, gscene, osc = c5_pair
    gp2 = GpuPlanner(robot, path_optimality_threshold=-np.inf)
    gp2.set_scene(gscene)
    pairs = scenes.random_queries(sc, 8, seed=7, check=lambda q: bool(gp2.check_configs([q])[0]))
    assert len(pairs) == 8
    qs = [GpuPlanner.make_query(s, g, sc.env_x, sc.env_y, samples=1_000_000, seed=1, query_id=k)
          for k, (s, g) in enumerate(pairs)]
    rs = gp2.plan_batch(qs)
    orc = O.Oracle(orobot, osc)
    for k, ((s, g), r) in enumerate(zip(pairs, rs)):
        o = orc.plan(s, g, env_x=sc.env_x, env_y=sc.env_y, max_checked=1_000_000, seed=1, query=k,
                     opt_thresh=-np.inf)
        _same_query_result(r, o)


def test_reference_call_sequence():
    """squirrel_8dof_planner.cpp:1221-1248 through the BiRRTstarPlanner mirror."""
    sc = scenes.box_room()
    p = BiRRTstarPlanner(seed=3)
    p.initialize("robotino_robot")
    p.setOctree(sc.keys, resolution=sc.res)
    p.setDisabledLinkMapCollisions([])
    p.reset_planner_and_config()
    p.setPlanningSceneInfo(list(sc.env_x), list(sc.env_y), "scenario")
    assert p.init_planner(sc.start, sc.goal, 1, True, True)
    assert p.run_planner(1, 0, 300, False, 0.0, 0)
    traj = p.getJointTrajectoryRef()
    assert len(traj) > 2 and traj[0] == list(sc.start)
    assert p.isConfigValid(sc.start, True, True)
    assert not p.init_planner([5.05, 0.0, 0.0] + scenes.ARM_FOLDED, sc.goal, 1, True, True)
    # time budget (the node's flag_iter_or_time = 1)
    assert p.init_planner(sc.start, sc.goal, 1, True, True)
    ok = p.run_planner(1, 1, 0.5, False, 0.0, 1)
    assert ok and p.stats["time_total"] <= 1.5


# ------------------------------------------------------------------------------------------ fold / unfold (§8f)
def test_check_sequence_fold_keyframes(gp, orobot):
    """The node's fold / unfold loops (squirrel_8dof_planner.cpp:759-784, 814-823): normalized folding keyframes
    (60-67) copied into robot poses, first invalid pose from one batched check, on the reference's room3.ot map
    with the node's floor; checked against the oracle's per-pose validity."""
    from oracle import trajectory as OT
    from squirrel_motion_planner_amd.planner import normalize_trajectory
    kf = np.load(os.path.join(GOLD, "folding_poses_tuw-robotino2.npz"))["keyframes"]
    arm = normalize_trajectory(kf, [0.08] * 5)
    assert np.array_equal(arm, np.array(OT.normalize_trajectory(kf.tolist(), [0.08] * 5)))
    fc = (0.0, 0.0)
    gs = Scene.from_ot(open(os.path.join(GOLD, "room3.ot"), "rb").read(), floor_center=fc)
    keys = np.concatenate([np.load(os.path.join(GOLD, "room3_keys.npz"))["keys"].astype(np.int64),
                           scenes.floor_keys(fc, 0.05, 3.0)])
    gp.set_scene(gs)
    gp.set_disabled_map_links([])
    orc = O.Oracle(orobot, O.OracleScene(keys, 0.05))
    # every keyframe, untrimmed.  The stowed end of the trajectory (the tuw file's first keyframes, arm_joint2 2.26 rad)
    # rests the fingers inside the front shell's exact box of robotino_plan.urdf (:323-329), so under this collision
    # model (that URDF's primitives + the finger covers of squirrel-hand.dae) they are in self-collision.  Whether the
    # reference agrees is UNPINNED: the deployed launch file does not load robotino_plan.urdf (planner.launch:14 is
    # commented out), FCL is absent, and the reference ships no vectors for it.  What is asserted is GPU == oracle, pose
    # by pose and pair by pair.
    poses0 = np.array([[0.0, 0.0, 0.0] + list(a) for a in arm])
    ok_self = orc.check_configs(poses0, True, False)
    assert ok_self[0] == 0 and ok_self[-1] == 1, ok_self
    assert np.array_equal(gp.check_configs(poses0, True, False), ok_self)
    pairs, _ = gp.get_collisions(poses0[0])
    assert pairs == orc.collisions(poses0[0])[0]
    assert ("hand_middle_finger_upper_link", "shell_base_link_front") in pairs
    rng = np.random.default_rng(4)
    firsts = []
    for k in range(48):
        base = [rng.uniform(-3.0, 3.0), rng.uniform(-3.0, 3.0), rng.uniform(-np.pi, np.pi)]
        poses = np.array([base + list(a) for a in (arm if k % 2 else arm[::-1])])
        flags = (k % 4 != 1, k % 3 != 0)   # some sequences map-only or self-only
        first = gp.check_sequence(poses, *flags)
        ov = orc.check_configs(poses, *flags)
        bad = np.flatnonzero(ov == 0)
        assert first == (bad[0] if len(bad) else -1), (k, first, bad[:3])
        firsts.append((first, poses, flags))
    assert any(f < 0 for f, _, _ in firsts) and any(f >= 0 for f, _, fl in firsts if not fl[0]), \
        [(f, fl) for f, _, fl in firsts]
    # a collision in the middle of a sequence: valid poses (the unfolded tail, self and map free), then a colliding one
    tail = int(np.flatnonzero(ok_self == 0)[-1]) + 1
    good = [p[-(len(arm) - tail):] for f, p, fl in firsts if fl == (True, True) and f >= 0 and p[-1][3] == arm[-1][0]]
    good = [g for g in good if orc.check_configs(g).all()]
    assert good
    seq = np.concatenate([good[0], poses0[:1] + np.array([good[0][0][0], good[0][0][1], good[0][0][2]] + [0.0] * 5),
                          good[-1]])
    want = orc.check_configs(seq)
    assert want[:len(good[0])].all() and not want[len(good[0])]
    assert gp.check_sequence(seq) == len(good[0])
    assert gp.check_sequence(np.zeros((0, 8))) == -1


# ------------------------------------------------------------------------------------------ C1 as SURVEY specifies it
def test_c1_survey_start_is_in_self_collision(gp, orobot):
    """SURVEY C1's start -- the first tuw folding keyframe -- puts the fingers inside the front shell's exact box of
    robotino_plan.urdf (:323-329; the finger meshes of squirrel-hand.dae enter it too, tools/gen_robot_model.py
    validate): under this collision model init_planner refuses it (birrt_star.cpp:353-357) on the GPU and in the oracle
    alike, with the same collision listing.  The reference's own behaviour for this start is UNPINNED: its deployed launch
    file does not load robotino_plan.urdf (planner.launch:14 is commented out) and FCL is absent here.  The planning C1
    cases start from pose_folded_arm instead (scenes.empty_room)."""
    sc = scenes.empty_room(stowed=True)
    gs = Scene.from_keys(sc.keys, sc.res)
    gp.set_scene(gs)
    gp.set_disabled_map_links([])
    orc = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res))
    o = orc.plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=100, seed=1)
    assert o["status"] == -2
    r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=100, seed=1))
    assert r["status"] == L.SMP_ERR_START_INVALID
    pairs, links = gp.get_collisions(sc.start)
    assert (pairs, links) == orc.collisions(sc.start)
    assert all("shell_base_link_front" in p or "base_body_link" in p for p in pairs) and pairs
    p = BiRRTstarPlanner()
    p.initialize()
    p.setOctree(sc.keys, resolution=sc.res)
    assert not p.init_planner(sc.start, sc.goal, 1, True, True)
    assert p.init_planner(sc.start, sc.goal, 1, False, True)  # without the self check the start is free


# ------------------------------------------------------------------------------------------ distributed scans
@pytest.mark.parametrize("scan_min,helpers,scouts,iters,seed", [(64, 0, 1, 3000, 5), (64, 63, 0, 1500, 9),
                                                               (600, 0, 1, 3000, 13)])
def test_distributed_scans_parity(orobot, robot, monkeypatch, scan_min, helpers, scouts, iters, seed):
    """Nearest and near scans split over the helper workgroups (DESIGN.md "Scans of large trees"), forced onto small
    trees (SMP_SCAN_MIN): trees, costs, counters and path bit for bit against the oracle."""
    monkeypatch.setenv("SMP_SCAN_MIN", str(scan_min))
    gp2 = GpuPlanner(robot, helpers=helpers, scout=scouts, path_optimality_threshold=-np.inf)
    sc, gscene, osc = scene_pair("c2")
    gp2.set_scene(gscene)
    r = gp2.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=iters, seed=seed))
    o = O.Oracle(orobot, osc).plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=iters, seed=seed,
                                   opt_thresh=-np.inf)
    assert max(r["nodes_start"], r["nodes_goal"]) > scan_min
    assert_same_run(gp2, r, o)


def test_large_tree_run_matches_golden(robot):
    """One C2 query for 1e5 iterations (trees of ~50k nodes per side, the distributed scans at the default split)
    against the committed oracle run (tests/golden/make_large_golden.py): counters, c_best, both trees' SHA-256
    digests and the path."""
    import hashlib
    g = np.load(os.path.join(GOLD, "plan_c2_1e5.npz"))
    gp2 = GpuPlanner(robot, path_optimality_threshold=-np.inf)
    sc, gscene, osc = scene_pair("c2")
    gp2.set_scene(gscene)
    r = gp2.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=int(g["iterations"]),
                                       seed=int(g["seed"])))
    dig = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert r["iterations"] == int(g["iterations"]) and r["first_solution_iter"] == int(g["first_iter"])
    assert r["configs_checked"] == int(g["checked"]) and r["configs_valid"] == int(g["valid"])
    assert r["nodes_start"] == int(g["n_start"]) and r["nodes_goal"] == int(g["n_goal"])
    assert [r["rewires_start"], r["rewires_goal"]] == g["rewires"].tolist()
    assert r["cost_best"] == g["cost"].tolist()
    for w, name in ((0, "start"), (1, "goal")):
        par, conf, cost = gp2.tree(w)
        assert dig(par) == str(g[name + "_parent_sha"]), name
        assert dig(conf) == str(g[name + "_conf_sha"]), name
        assert dig(cost) == str(g[name + "_cost_sha"]), name
    assert np.array_equal(r["path"], g["path"])


@pytest.mark.parametrize("n1,n2", [(3000, 3600), (20000, 20300), (300000, 300200)])
def test_oracle_continues_the_gpu_state(gp, orobot, n1, n2):
    """The oracle continued from the GPU planner's state after n1 iterations (GpuPlanner.export_state ->
    Oracle.resume: both trees with their child order and in-edges, the loop scalars) plans exactly the GPU's own run of
    n2 iterations: the GPU's state is the reference loop's state at n1, and the large-tree CPU timing
    (bench.py cpu_window) resumes the CPU from the GPU's trees.  The 3e5 case (trees of ~160k / ~140k nodes) runs the
    distributed scans' fp32-prefiltered slices (DESIGN.md "fp32 prefilter") where they are built for: every nearest
    (first strict minimum, BS:4076-4133) and near set (radius test, BS:4272-4324) of its last 200 iterations must equal
    the oracle's fp64 scans for the trees, costs and path to match."""
    sc, gscene, osc = scene_pair("c2")
    gp.set_scene(gscene)
    gp.set_disabled_map_links([])
    kw = dict(env_x=sc.env_x, env_y=sc.env_y, seed=7, opt_thresh=-math.inf)
    gpl = GpuPlanner(path_optimality_threshold=-math.inf)
    gpl.set_scene(gscene)
    gpl.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=n1, seed=7))
    st = gpl.export_state()
    r = gpl.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=n2, seed=7))
    o = O.Oracle(orobot, osc).resume(sc.start, sc.goal, st, max_iter=n2, **kw)
    assert o["iterations"] == r["iterations"] == n2
    assert o["checked"] == r["configs_checked"] and o["valid"] == r["configs_valid"]
    assert o["n_start"] == r["nodes_start"] and o["n_goal"] == r["nodes_goal"]
    assert o["cost"] == list(r["cost_best"])
    for which, name in ((0, "start"), (1, "goal")):
        par, conf, cost = gpl.tree(which)
        assert np.array_equal(par, o[name + "_parent"])
        assert np.array_equal(conf, o[name + "_conf"]) and np.array_equal(cost, o[name + "_cost"])
    assert np.array_equal(r["path"], o["path"])
