"""Failure reporting and budget semantics of smp_plan / smp_plan_batch (GPU).

The reference returns bool and logs (birrt_star.cpp:338-362, 1405); through the C ABI every query's status says
what happened, and a call that fails underneath (a HIP error) never reads as a success: each result carries the
error status and the Python binding raises.
"""
import math
import time

import numpy as np
import pytest

from squirrel_motion_planner_amd import _lib as L
from squirrel_motion_planner_amd import scenes
from squirrel_motion_planner_amd.planner import GpuPlanner, Robot, Scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2():
    sc = scenes.box_room()
    return sc, Scene.from_keys(sc.keys, sc.res)


def test_allocation_failure_raises(c2):
    sc, scene = c2
    gp = GpuPlanner(Robot(), node_capacity=1 << 40)  # ~2e14 bytes of trees: hipMalloc fails
    gp.set_scene(scene)
    with pytest.raises(L.SmpError) as e:
        gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=10, seed=1))
    assert e.value.status == L.SMP_ERR_HIP
    # the planner stays usable after a failed call
    gp.params.node_capacity = 0
    L.check(L.lib().smp_planner_set_params(gp.h, gp.params))
    r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=50, seed=1))
    assert r["status"] in (L.SMP_OK, L.SMP_ERR_NO_SOLUTION)


def test_unknown_budget_kind_is_an_argument_error(c2):
    sc, scene = c2
    gp = GpuPlanner(Robot())
    gp.set_scene(scene)
    good = GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=50, seed=1)
    bad = GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=50, seed=1)
    bad.budget_kind = 7
    t = time.perf_counter()
    r_good, r_bad = gp.plan_batch([good, bad])
    assert time.perf_counter() - t < 30
    assert r_bad["status"] == L.SMP_ERR_ARG and r_bad["iterations"] == 0
    assert r_good["status"] in (L.SMP_OK, L.SMP_ERR_NO_SOLUTION) and r_good["iterations"] == 50


def test_seconds_budget_counts_from_the_call(c2):
    sc, scene = c2
    gp = GpuPlanner(Robot(), path_optimality_threshold=-math.inf)
    gp.set_scene(scene)
    q = GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, seconds=0.05, seed=1)
    gp.plan(q)  # first call: allocations
    t = time.perf_counter()
    r = gp.plan(q)
    wall = time.perf_counter() - t
    assert r["status"] == L.SMP_OK and r["iterations"] > 0
    # the device deadline is set when the kernel records the start, from the budget left at launch
    assert r["time_total"] <= 0.05 + 0.01, r["time_total"]
    assert wall < 0.05 + 0.5


@pytest.mark.parametrize("cap", [9000, 4000])
def test_seconds_budget_keeps_the_path_when_a_tree_fills(c2, cap):
    sc, scene = c2
    # two via chains of cap/8 nodes each are held back for one iteration: the run stops once a tree holds about
    # three quarters of the capacity, with the best path so far
    gp = GpuPlanner(Robot(), path_optimality_threshold=-math.inf, node_capacity=cap)
    gp.set_scene(scene)
    r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, seconds=20.0, seed=1))
    assert r["status"] == L.SMP_OK, r["status"]
    assert len(r["path"]) > 0
    margin = 2 * max(64, min(4096, cap // 8)) + 4
    n = max(r["nodes_start"], r["nodes_goal"])
    assert n + margin > cap and n > cap // 2, (n, cap)
    assert r["iterations"] > 100
    assert r["time_total"] < 5.0


def test_oversubscribed_helpers_are_clamped(c2):
    # a helper request beyond the co-resident capacity (occupancy x CUs) falls back to the automatic count: every
    # helper has to be running for the leader's jobs not to wait out its tile timeout
    sc, scene = c2
    q = lambda: GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, samples=200_000, seed=3)
    auto = GpuPlanner(Robot(), path_optimality_threshold=-math.inf)
    auto.set_scene(scene)
    over = GpuPlanner(Robot(), path_optimality_threshold=-math.inf, helpers=1000)
    over.set_scene(scene)
    auto.plan(q()), over.plan(q())  # first-call allocation
    ra, ro = auto.plan(q()), over.plan(q())
    assert 0 < ro["helpers"] <= ra["helpers"], (ro["helpers"], ra["helpers"])
    for k in ("iterations", "configs_checked", "nodes_start", "nodes_goal", "cost_best"):
        assert ro[k] == ra[k], k
    assert ro["time_total"] < 2.0 * ra["time_total"] + 0.01, (ro["time_total"], ra["time_total"])


def test_abandoned_launch_drains_on_the_abort_word(c2, monkeypatch):
    """A call whose wait for its launch times out returns SMP_ERR_HIP and marks the planner busy (its buffers are still in
    use); it also sets the host-mapped abort word that every leader polls every ABORT_EVERY iterations, so the launch
    ends within a few milliseconds instead of running to the end of its budget.  Here the wait is cut to 0.1 s of a 5 s
    budget (SMP_WAIT_SLACK_S = -19.9: 4 x 5 s - 19.9 s): the planner is usable again well before the budget's end, and
    plans as before."""
    sc, scene = c2
    gp = GpuPlanner(Robot(), path_optimality_threshold=-math.inf)
    gp.set_scene(scene)
    ref = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=300, seed=2))
    monkeypatch.setenv("SMP_WAIT_SLACK_S", "-19.9")
    t = time.perf_counter()
    with pytest.raises(L.SmpError) as e:
        gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, seconds=5.0, seed=1))
    assert e.value.status == L.SMP_ERR_HIP
    monkeypatch.delenv("SMP_WAIT_SLACK_S")
    r = None
    while time.perf_counter() - t < 4.0:
        try:
            r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=300, seed=2))
            break
        except L.SmpError as busy:
            assert busy.status == L.SMP_ERR_HIP
            time.sleep(0.01)
    drained = time.perf_counter() - t
    assert r is not None and drained < 1.0, drained
    for k in ("status", "iterations", "configs_checked", "nodes_start", "nodes_goal"):
        assert r[k] == ref[k], k
    assert np.array_equal(r["path"], ref["path"])
