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


def test_early_ask_records_past_the_first_solution(c2, orobot, monkeypatch):
    """SMP_EARLY_ASK=1: post-solution scouts are asked for iteration k + 2 at the start of iteration k and build their
    records while the leader still rewires (DESIGN.md "Where the iteration's time goes").  The leader takes a record's
    nearest node -- its configuration and costs -- from the record instead of reloading it (iteration(), the staged
    record), which is exact only if the record's rewire count and the rwb / rwe wait reject every record built on costs
    a rewire has since changed.  Planned 3000 iterations (first solution near iteration 120, then ~2900 iterations of
    rewires), the run must equal the oracle's bit for bit, as must the default mode."""
    from oracle import oracle as O
    sc, scene = c2
    osc = O.OracleScene(sc.keys, sc.res)
    o = O.Oracle(orobot, osc).plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=3000, seed=1,
                                   opt_thresh=-math.inf)
    assert 0 <= o["first_iter"] < 1000
    for env in ({"SMP_EARLY_ASK": "1"}, {"SMP_EARLY_ASK": "0"}):
        for k in ("SMP_PRE_REFRESH", "SMP_PRE_COMMIT", "SMP_EARLY_ASK"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        gp = GpuPlanner(path_optimality_threshold=-math.inf)
        gp.set_scene(scene)
        r = gp.plan(GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=3000, seed=1))
        assert r["iterations"] == o["iterations"] and r["first_solution_iter"] == o["first_iter"], env
        assert r["configs_checked"] == o["checked"] and r["configs_valid"] == o["valid"], env
        assert r["nodes_start"] == o["n_start"] and r["nodes_goal"] == o["n_goal"], env
        assert r["rewires_start"] == o["rewires_start"] and r["rewires_goal"] == o["rewires_goal"], env
        for w, name in ((0, "start"), (1, "goal")):
            par, conf, cost = gp.tree(w)
            assert np.array_equal(par, o[name + "_parent"]), (env, name)
            assert np.array_equal(conf, o[name + "_conf"]) and np.array_equal(cost, o[name + "_cost"]), (env, name)
        assert r["cost_best"] == o["cost"], env
        assert np.array_equal(r["path"], o["path"]), env
