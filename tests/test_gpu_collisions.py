"""getCollisions (birrt_star.cpp:6910-6914 -> collision_checker.hpp:123-132, 594-630) on the GPU
(`smp_get_collisions`, one wavefront) against the oracle's restatement (smp_oracle.cpp orc_collisions), as link names:
the overlapping self pairs in the model's pair order and the links touching the map in name order, disabled links
included (getMapCollisions ignores the disabled flag)."""
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle import oracle as O
from squirrel_motion_planner_amd import scenes
from squirrel_motion_planner_amd.planner import BiRRTstarPlanner, GpuPlanner, Scene

pytestmark = pytest.mark.gpu

MODEL = os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")


def probes(sc, n, seed):
    """Random base poses over the map and arm poses over the joint ranges, plus the scene's start and goal."""
    rng = np.random.default_rng(seed)
    lo, hi = [-1.2, -1.7, -1.8, -2.4, -2.9], [1.5, 2.6, 1.8, 2.4, 2.9]  # arm limits
    q = np.column_stack([rng.uniform(sc.env_x[0], sc.env_x[1], n), rng.uniform(sc.env_y[0], sc.env_y[1], n),
                         rng.uniform(-np.pi, np.pi, n)] + [rng.uniform(lo[j], hi[j], n) for j in range(5)])
    return np.vstack([np.asarray(sc.start)[None], np.asarray(sc.goal)[None], q])


@pytest.mark.parametrize("scene_name", ["box_room", "narrow_passage"])
def test_get_collisions_matches_oracle(scene_name):
    sc = getattr(scenes, scene_name)()
    gp = GpuPlanner(device=0)
    gp.set_scene(Scene.from_keys(sc.keys, sc.res))
    orc = O.Oracle(O.OracleRobot(MODEL), O.OracleScene(sc.keys, sc.res))
    Q = probes(sc, 300, 11)
    valid = orc.check_configs(Q)
    n_self = n_map = 0
    for q, v in zip(Q, valid):
        got = gp.get_collisions(q)
        want = orc.collisions(q)
        assert got == want, (q.tolist(), got, want)
        assert (len(got[0]) + len(got[1]) == 0) == bool(v)  # isInCollision iff something is listed
        n_self += len(got[0]) > 0
        n_map += len(got[1]) > 0
    assert n_self > 5 and n_map > 20  # the probes exercise both lists


def test_get_collisions_lists_disabled_links_and_appends():
    sc = scenes.box_room()
    p = BiRRTstarPlanner()
    p.initialize("robotino_robot")
    p._gpu.set_scene(Scene.from_keys(sc.keys, sc.res))
    orc = O.Oracle(O.OracleRobot(MODEL), O.OracleScene(sc.keys, sc.res))
    Q = probes(sc, 200, 5)
    hit = next(q for q in Q if orc.collisions(q)[1])
    links = orc.collisions(hit)[1]
    p.setDisabledLinkMapCollisions(links)
    self_c, map_c = [("x", "y")], ["z"]
    p.getCollisions(list(hit), self_c, map_c)
    want = orc.collisions(hit)
    assert self_c == [("x", "y")] + want[0] and map_c == ["z"] + want[1]
    # every map-colliding link is disabled: the planner's map check passes while the listing still names them
    assert p.isConfigValid(list(hit), False, True)
