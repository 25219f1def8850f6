"""Writes tests/golden/folding_poses_tuw-robotino2.npz: the reference's folding keyframes (5 arm joints each,
squirrel_8dof_planner/config/folding_poses_tuw-robotino2.yaml, loaded by the node at squirrel_8dof_planner.cpp:48-67)
as a data fixture, so GPU tests do not read /root/reference."""
import os

import numpy as np
import yaml

SRC = "/root/reference/squirrel_8dof_planner/config/folding_poses_tuw-robotino2.yaml"

if __name__ == "__main__":
    with open(SRC) as f:
        v = yaml.safe_load(f)["trajectory_folding_arm"]
    kf = np.asarray(v, np.float64).reshape(-1, 5)
    np.savez(os.path.join(os.path.dirname(os.path.abspath(__file__)), "folding_poses_tuw-robotino2.npz"), keyframes=kf)
    print(kf.shape)
