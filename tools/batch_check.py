import math, os, sys
import numpy as np
sys.path.insert(0, "/root/repo")
from oracle import oracle as O
from squirrel_motion_planner_amd import scenes
from squirrel_motion_planner_amd.planner import GpuPlanner, Scene
sc = scenes.box_room()
gp = GpuPlanner()
gp.set_scene(Scene.from_keys(sc.keys, sc.res))
orob = O.OracleRobot("/root/repo/squirrel_motion_planner_amd/data/robotino_model.json")
orc = O.Oracle(orob, O.OracleScene(sc.keys, sc.res))
for rep in range(3):
    qs = [GpuPlanner.make_query(sc.start, sc.goal, sc.env_x, sc.env_y, iterations=150, seed=s, query_id=s) for s in range(4)]
    batch = gp.plan_batch(qs)
    for s, b in enumerate(batch):
        o = orc.plan(sc.start, sc.goal, env_x=sc.env_x, env_y=sc.env_y, max_iter=150, seed=s, query=s)
        single = gp.plan(qs[s])
        print("rep %d q%d: batch checked %d first %d | single %d first %d | oracle %d first %d" % (
            rep, s, b["configs_checked"], b["first_solution_iter"], single["configs_checked"], single["first_solution_iter"],
            o["checked"], o["first_iter"]), flush=True)
