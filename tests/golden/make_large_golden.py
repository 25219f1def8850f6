"""Writes tests/golden/plan_c2_1e5.npz: one C2 query planned by the oracle for 1e5 iterations (the large-tree regime
of SURVEY.md 8d: trees of ~60k nodes per side).  The trees themselves are stored as SHA-256 digests of the parent
arrays and configurations (the fixture stays small); the counters, c_best, the cost rows' last value and the path are
stored as they are.  Takes ~15 min on one core (oracle/smp_oracle.cpp)."""
import hashlib
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from squirrel_motion_planner_amd import scenes  # noqa: E402

ITERS, SEED = 100000, 7


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


if __name__ == "__main__":
    sc = scenes.box_room()
    rob = O.OracleRobot(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json"))
    orc = O.Oracle(rob, O.OracleScene(sc.keys, sc.res))
    t = time.time()
    r = orc.plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=ITERS, seed=SEED, opt_thresh=-math.inf)
    print("planned in %.0f s" % (time.time() - t), r["status"], r["iterations"], r["n_start"], r["n_goal"], r["checked"])
    np.savez_compressed(os.path.join(HERE, "plan_c2_1e5.npz"), iterations=r["iterations"], seed=SEED,
                        status=r["status"], first_iter=r["first_iter"], last_iter=r["last_iter"], checked=r["checked"],
                        valid=r["valid"], n_start=r["n_start"], n_goal=r["n_goal"], cost=np.array(r["cost"]),
                        rewires=np.array([r["rewires_start"], r["rewires_goal"]]),
                        conn=np.array([r["conn_start"], r["conn_b"], r["conn_a"]]), path=r["path"],
                        start_parent_sha=digest(r["start_parent"]), goal_parent_sha=digest(r["goal_parent"]),
                        start_conf_sha=digest(r["start_conf"]), goal_conf_sha=digest(r["goal_conf"]),
                        start_cost_sha=digest(r["start_cost"]), goal_cost_sha=digest(r["goal_cost"]),
                        t_total=r["t_total"])
