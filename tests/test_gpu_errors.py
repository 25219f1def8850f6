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


def test_seconds_budget_keeps_the_path_when_a_tree_fills(c2):
    sc, scene = c2
    # 8196 nodes are held back for one iteration's via chains: the run stops once a tree holds ~800 nodes
    gp = GpuPlanner(Robot(), path_optimality_threshold=-math.inf, node_capacity=9000)
    gp.set_scene(scene)
    r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, seconds=20.0, seed=1))
    assert r["status"] == L.SMP_OK, r["status"]
    assert len(r["path"]) > 0
    assert max(r["nodes_start"], r["nodes_goal"]) + 8196 > 9000
    assert r["time_total"] < 5.0
