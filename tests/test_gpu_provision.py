"""Provisioning edge cases: a per-XCD helper cap that leaves fewer than four helpers must also
drop the scouts (a scout without helpers has no worker for its tiles), so planning still finishes and answers exactly
as with the default provisioning."""
import math

import numpy as np
import pytest

from squirrel_motion_planner_amd import scenes
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene

pytestmark = pytest.mark.gpu


def _plan(margin, monkeypatch):
    if margin is None:
        monkeypatch.delenv("SMP_XCD_MARGIN", raising=False)
    else:
        monkeypatch.setenv("SMP_XCD_MARGIN", str(margin))
    sc = scenes.box_room()
    gp = GpuPlanner(path_optimality_threshold=-math.inf)
    gp.set_scene(Scene.from_keys(sc.keys, sc.res))
    return gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=400, seed=5))


@pytest.mark.parametrize("margin", [26, 29, 64])
def test_xcd_cap_below_four_helpers_finishes_with_same_result(margin, monkeypatch):
    ref = _plan(None, monkeypatch)
    got = _plan(margin, monkeypatch)
    for k in ("status", "iterations", "configs_checked", "configs_valid", "nodes_start", "nodes_goal",
              "first_solution_iter", "nn_nodes_scanned", "near_nodes_scanned"):
        assert got[k] == ref[k], (margin, k, got[k], ref[k])
    assert np.array_equal(np.asarray(got["cost_best"]), np.asarray(ref["cost_best"]))
    assert np.array_equal(np.asarray(got["path"]), np.asarray(ref["path"]))
    assert got["helpers"] < ref["helpers"]
