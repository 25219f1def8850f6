"""Pre-solution records are speculation only: whether a scout restarts its pass on the leader's newer tree sizes
(SMP_PRE_REFRESH, DESIGN.md "Pre-solution refresh") or no record is committed at all (SMP_PRE_COMMIT=0: every
iteration runs the full path), the planner answers bit for bit the same.  A refreshed pass reads nodes the leader
stored after the scout's CU cached their lines; a stale copy would show here as a different tree."""
import math

import numpy as np
import pytest

from squirrel_motion_planner_amd import scenes
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene

pytestmark = pytest.mark.gpu

KEYS = ("status", "iterations", "configs_checked", "configs_valid", "nodes_start", "nodes_goal", "first_solution_iter")


@pytest.fixture(scope="module")
def c2():
    sc = scenes.box_room()
    return sc, Scene.from_keys(sc.keys, sc.res)


def _plan(c2, env, seed, monkeypatch):
    for k in ("SMP_PRE_REFRESH", "SMP_PRE_COMMIT"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc, scene = c2
    gp = GpuPlanner(path_optimality_threshold=-math.inf)
    gp.set_scene(scene)
    return gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=250, seed=seed))


@pytest.mark.parametrize("seed", [1, 6001, 10001])
def test_refreshed_records_answer_as_the_full_path(c2, seed, monkeypatch):
    ref = _plan(c2, {"SMP_PRE_COMMIT": "0"}, seed, monkeypatch)
    for env in ({"SMP_PRE_REFRESH": "0"}, {}, {"SMP_PRE_REFRESH": "3"}):
        got = _plan(c2, env, seed, monkeypatch)
        for k in KEYS:
            assert got[k] == ref[k], (env, k, got[k], ref[k])
        assert np.array_equal(np.asarray(got["cost_best"]), np.asarray(ref["cost_best"]))
        assert np.array_equal(np.asarray(got["path"]), np.asarray(ref["path"]))
