"""Regenerates the committed fixtures in tests/golden/ (run here, where /root/reference exists).

  room{3,4,5}_keys.npz  occupied leaf keys of the reference octomaps squirrel_8dof_planner/config/room*.bt,
                        decoded by oracle/octomap_bt.py (independent reader), plus the source sha256
  plan_*.npz            seeded oracle planner runs (trees, costs, paths, stats) that pin the oracle itself
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import octomap_bt, oracle as O  # noqa: E402
from squirrel_motion_planner_amd import scenes  # noqa: E402

REF = "/root/reference/squirrel_8dof_planner/config"

PLAN_CASES = {
    # name: (scene factory, planner kwargs)
    "c1_direct": (scenes.empty_room, dict(max_iter=50, seed=1)),
    "c2_boxes_300": (scenes.box_room, dict(max_iter=300, seed=3)),
    "c2_boxes_yaml": (scenes.box_room, dict(max_iter=200, seed=5, near_r=1.5, step=0.6)),
    "c4_passage": (scenes.narrow_passage, dict(max_iter=400, seed=2)),
}


def rooms():
    for r in ("room3", "room4", "room5"):
        raw = open(os.path.join(REF, r + ".bt"), "rb").read()
        res, keys = octomap_bt.read_bt(raw)
        np.savez_compressed(os.path.join(HERE, r + "_keys.npz"), keys=keys.astype(np.uint16), res=res,
                            sha256=hashlib.sha256(raw).hexdigest())
        print(r, len(keys))


def plan_case(name):
    mk, kw = PLAN_CASES[name]
    sc = mk()
    rob = O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json"))
    orc = O.Oracle(rob, O.OracleScene(sc.keys, sc.res))
    r = orc.plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, **kw)
    return sc, r


def plans():
    for name in PLAN_CASES:
        sc, r = plan_case(name)
        np.savez_compressed(os.path.join(HERE, "plan_%s.npz" % name), status=r["status"], path=r["path"],
                            start_parent=r["start_parent"], goal_parent=r["goal_parent"],
                            start_cost=r["start_cost"], goal_cost=r["goal_cost"], start_conf=r["start_conf"],
                            goal_conf=r["goal_conf"], cost=np.array(r["cost"]), checked=r["checked"],
                            valid=r["valid"], iterations=r["iterations"], first_iter=r["first_iter"])
        print(name, r["status"], r["iterations"], r["first_iter"], len(r["start_parent"]), len(r["goal_parent"]),
              r["checked"], r["cost"])


if __name__ == "__main__":
    if os.path.isdir(REF):
        rooms()
    plans()
