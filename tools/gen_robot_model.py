#!/usr/bin/env python3
"""Generate squirrel_motion_planner_amd/data/robotino_model.json from the reference robot description.

Run HERE (where /root/reference exists); the JSON is committed so the GPU box never needs the reference.

What it derives (all numbers are plain fp64, written with repr() so they round-trip exactly):
  * the 12-segment planning chain base_link_origin -> hand_wrist_link (robotino_plan.srdf:4-6) with
    KDL segment semantics (kdl_parser: f_tip = joint.pose(0)^-1 * F_origin; kdl segment.cpp), used by the
    end-effector FK of the sampler (kdl_kuka_model.cpp:278-305);
  * the 39-link collision tree in KDL-tree DFS order (collision_checker.hpp:195-261): movable links of the
    8 planning joints keep (axis, origin) only (joint->pose(q), collision_checker.hpp:527-528), every other
    link keeps its frame-to-tip times the collision-origin adjust, which propagates to children
    (collision_checker.hpp:329-336 + 530 -- the reference quirk, reproduced);
  * joint limits cast through float exactly like kdl_kuka_model.cpp:165-190 (continuous -> +-(float)M_PI);
  * the 230 SRDF-enabled self-collision link pairs (collision_checker.hpp:353-389, parseSRDF 395-421);
  * a sphere decomposition of every collision link.  The reference collides FCL meshes/primitives; the
    meshes (package://robotino_description) are absent from the reference tree, so the geometry is a
    documented approximation (DESIGN.md "Collision model").  Primitive links (box/cylinder) are covered
    from their URDF dimensions; mesh links use hand-fitted spheres along the kinematic offsets.

The generator validates the model: every arm keyframe of the reference folding trajectory
(squirrel_8dof_planner/config/parameters.yaml:45-69) must be self-collision free with the base at the origin.
"""
import itertools
import json
import math
import os
import sys
import xml.etree.ElementTree as ET

import numpy as np

REF = "/root/reference/squirrel_8dof_planner/config"
OUT = os.path.join(os.path.dirname(__file__), "..", "squirrel_motion_planner_amd", "data", "robotino_model.json")

PLAN_JOINT_LINKS = ["base_x_link", "base_y_link", "base_theta_link", "arm_link1", "arm_motor2",
                    "arm_link3", "arm_link4", "arm_link5"]  # collision_checker.hpp:216-255


# ---------------------------------------------------------------- KDL-style frame algebra (fp64, no FMA)
def rot_mul(a, b):
    return [a[r * 3 + 0] * b[0 * 3 + c] + a[r * 3 + 1] * b[1 * 3 + c] + a[r * 3 + 2] * b[2 * 3 + c]
            for r in range(3) for c in range(3)]


def rot_vec(a, v):
    return [a[r * 3 + 0] * v[0] + a[r * 3 + 1] * v[1] + a[r * 3 + 2] * v[2] for r in range(3)]


def frame_mul(f1, f2):
    R1, p1 = f1
    R2, p2 = f2
    mp = rot_vec(R1, p2)
    return (rot_mul(R1, R2), [mp[i] + p1[i] for i in range(3)])


IDENT = ([1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0], [0.0, 0.0, 0.0])


def quat_from_rpy(roll, pitch, yaw):  # urdfdom Rotation::setFromRPY + normalize
    phi, the, psi = roll / 2.0, pitch / 2.0, yaw / 2.0
    x = math.sin(phi) * math.cos(the) * math.cos(psi) - math.cos(phi) * math.sin(the) * math.sin(psi)
    y = math.cos(phi) * math.sin(the) * math.cos(psi) + math.sin(phi) * math.cos(the) * math.sin(psi)
    z = math.cos(phi) * math.cos(the) * math.sin(psi) - math.sin(phi) * math.sin(the) * math.cos(psi)
    w = math.cos(phi) * math.cos(the) * math.cos(psi) + math.sin(phi) * math.sin(the) * math.sin(psi)
    s = math.sqrt(x * x + y * y + z * z + w * w)
    if s == 0.0:
        return 0.0, 0.0, 0.0, 1.0
    return x / s, y / s, z / s, w / s


def rot_from_quat(x, y, z, w):  # KDL::Rotation::Quaternion
    x2, y2, z2, w2 = x * x, y * y, z * z, w * w
    return [w2 + x2 - y2 - z2, 2 * x * y - 2 * w * z, 2 * x * z + 2 * w * y,
            2 * x * y + 2 * w * z, w2 - x2 + y2 - z2, 2 * y * z - 2 * w * x,
            2 * x * z - 2 * w * y, 2 * y * z + 2 * w * x, w2 - x2 - y2 + z2]


def rot2(axis, angle):  # KDL::Rotation::Rot2 (generator-side only, libm sin/cos)
    ct, st = math.cos(angle), math.sin(angle)
    vt = 1 - ct
    m_vt_0, m_vt_1, m_vt_2 = vt * axis[0], vt * axis[1], vt * axis[2]
    m_st_0, m_st_1, m_st_2 = axis[0] * st, axis[1] * st, axis[2] * st
    m_vt_0_1, m_vt_0_2, m_vt_1_2 = m_vt_0 * axis[1], m_vt_0 * axis[2], m_vt_1 * axis[2]
    return [ct + m_vt_0 * axis[0], -m_st_2 + m_vt_0_1, m_st_1 + m_vt_0_2,
            m_st_2 + m_vt_0_1, ct + m_vt_1 * axis[1], -m_st_0 + m_vt_1_2,
            -m_st_1 + m_vt_0_2, m_st_0 + m_vt_1_2, ct + m_vt_2 * axis[2]]


def kdl_norm(v):  # KDL::Vector::Norm
    a0, a1, a2 = abs(v[0]), abs(v[1]), abs(v[2])
    def sq(x):
        return x * x
    if a0 >= a1:
        if a0 >= a2:
            if a0 == 0:
                return 0.0
            return a0 * math.sqrt(1 + sq(v[1] / v[0]) + sq(v[2] / v[0]))
        return a2 * math.sqrt(1 + sq(v[0] / v[2]) + sq(v[1] / v[2]))
    if a1 >= a2:
        return a1 * math.sqrt(1 + sq(v[0] / v[1]) + sq(v[2] / v[1]))
    return a2 * math.sqrt(1 + sq(v[0] / v[2]) + sq(v[1] / v[2]))


def frame_inverse(f):
    R, p = f
    Rt = [R[0], R[3], R[6], R[1], R[4], R[7], R[2], R[5], R[8]]
    mp = rot_vec(Rt, p)
    return (Rt, [-mp[0], -mp[1], -mp[2]])


def parse_floats(s, n=3, default=0.0):
    if s is None:
        return [default] * n
    return [float(t) for t in s.split()]


# ---------------------------------------------------------------- URDF -> KDL joint/segment model
class Joint:
    def __init__(self, el):
        self.name = el.get("name")
        self.type = el.get("type")
        self.parent = el.find("parent").get("link")
        self.child = el.find("child").get("link")
        o = el.find("origin")
        xyz = parse_floats(o.get("xyz") if o is not None else None)
        rpy = parse_floats(o.get("rpy") if o is not None else None)
        q = quat_from_rpy(*rpy)
        self.F = (rot_from_quat(*q), xyz)  # kdl_parser toKdl(urdf::Pose)
        ax = el.find("axis")
        self.axis_urdf = parse_floats(ax.get("xyz")) if ax is not None else [1.0, 0.0, 0.0]
        lim = el.find("limit")
        self.lower = float(lim.get("lower")) if lim is not None and lim.get("lower") else 0.0
        self.upper = float(lim.get("upper")) if lim is not None and lim.get("upper") else 0.0
        # kdl_parser toKdl(joint): axis rotated into the parent frame, normalised by the Joint ctor
        if self.type in ("revolute", "continuous", "prismatic"):
            a = rot_vec(self.F[0], self.axis_urdf)
            n = kdl_norm(a)
            self.axis = [a[0] / n, a[1] / n, a[2] / n]
        else:
            self.axis = [0.0, 0.0, 0.0]
        self.kdl_type = {"revolute": "RotAxis", "continuous": "RotAxis", "prismatic": "TransAxis"}.get(self.type, "None")

    def pose(self, q):  # KDL::Joint::pose
        if self.kdl_type == "RotAxis":
            return (rot2(self.axis, q), list(self.F[1]))
        if self.kdl_type == "TransAxis":
            return (list(IDENT[0]), [self.F[1][i] + self.axis[i] * q for i in range(3)])
        return (list(IDENT[0]), [0.0, 0.0, 0.0])

    def f_tip(self):  # KDL::Segment ctor: f_tip = joint.pose(0).Inverse() * F
        return frame_mul(frame_inverse(self.pose(0.0)), self.F)

    def frame_to_tip(self):  # Segment::getFrameToTip = joint.pose(0) * f_tip
        return frame_mul(self.pose(0.0), self.f_tip())


# Sphere covers of the mesh links, in each link's collision frame (the frame FCL places the mesh in).  The robotino
# meshes (package://robotino_description) are absent from the reference, so the base, arm and wrist covers are fitted
# by hand along the URDF's kinematic offsets; the kclhand links are fitted to the meshes of the reference's
# squirrel-hand.dae (tools/hand_spheres.py: every triangle inside a sphere).  Written to SPEC_OUT, the spheres_json input
# of smp_robot_create_urdf.
SPEC_OUT = os.path.join(os.path.dirname(__file__), "..", "squirrel_motion_planner_amd", "data", "robotino_spheres.json")
HAND_SPHERES = None


def sphere_spec():
    global HAND_SPHERES
    spec = {}
    # RobotinoBody: base cylinder, ~0.37 m diameter
    spec["base_body_link"] = [[x, y, 0.09, 0.085] for x in (-0.07, 0.07) for y in (-0.07, 0.07)]
    spec["shell_base_link"] = [[-0.20, 0.0, z, 0.09] for z in (0.36, 0.48, 0.60)]  # tower behind the arm column
    spec["door_link"] = [[-0.22, 0.0, 0.46, 0.05]]
    spec["arm_base_link"] = [[0.0, 0.0, 0.035, 0.05]]
    spec["arm_link1"] = [[0.0, 0.0, z, 0.045] for z in (0.07, 0.14, 0.20)]  # 0.25 m up to arm_joint2 (urdf:648)
    spec["arm_link2"] = [[0.0, 0.0, z, 0.045] for z in (0.03, 0.10)]  # 0.158 m up to arm_joint3 (urdf:697)
    spec["arm_link3"] = [[0.0, -0.03, 0.035, 0.04]]  # to (0,-0.057,0.065)
    spec["arm_link4"] = [[0.0, -0.014, 0.02, 0.035]]  # to (0,-0.027,0.035)
    spec["hand_wrist_link"] = [[0.0, 0.06, 0.0, 0.045]]  # wrist.stl (absent): hand extends along wrist +y
    spec["hand_cableCanal_link"] = [[0.0, 0.0, 0.0, 0.02]]  # cableCanalCollision.stl (absent)
    if HAND_SPHERES is None:
        import hand_spheres
        HAND_SPHERES, rep = hand_spheres.hand_spheres(os.path.join(REF, "squirrel-hand.dae"))
        for k, v in rep.items():
            print("hand cover %-32s %5d triangles -> %d spheres, max r %.4f m" % (k, v[0], len(HAND_SPHERES[k]), v[1]),
                  file=sys.stderr)
    spec.update(HAND_SPHERES)
    return spec


def f32(x):
    return float(np.float32(x))


def build_model():
    urdf = ET.parse(os.path.join(REF, "robotino_plan.urdf")).getroot()
    srdf = ET.parse(os.path.join(REF, "robotino_plan.srdf")).getroot()
    links = {l.get("name"): l for l in urdf.findall("link")}
    joints = [Joint(j) for j in urdf.findall("joint")]
    by_child = {j.child: j for j in joints}
    children = {}
    for j in sorted(joints, key=lambda j: j.name):  # urdf initTree iterates the joint map (sorted by name)
        children.setdefault(j.parent, []).append(j.child)
    roots = [n for n in links if n not in by_child]
    assert roots == ["base_link_origin"], roots

    # ---- planning chain (srdf group chain)
    chain_el = srdf.find("group").find("chain")
    base, tip = chain_el.get("base_link"), chain_el.get("tip_link")
    seq = []
    n = tip
    while n != base:
        seq.append(by_child[n])
        n = by_child[n].parent
    seq.reverse()
    chain = []
    qmin, qmax, jnames, jrev = [], [], [], []
    for j in seq:
        ft = j.f_tip()
        ent = {"name": j.child, "joint_name": j.name, "type": j.kdl_type, "axis": j.axis, "origin": j.F[1],
               "ftip_R": ft[0], "ftip_p": ft[1]}
        if j.kdl_type != "None":
            ent["joint"] = len(jnames)
            jnames.append(j.name)
            jrev.append(1 if j.kdl_type == "RotAxis" else 0)
            if j.type == "continuous":  # kdl_kuka_model.cpp:176-184 (stored through float)
                lo, hi = f32(-math.pi), f32(math.pi)
            else:
                lo, hi = f32(j.lower), f32(j.upper)
            qmin.append(lo)
            qmax.append(hi)
        else:
            ent["joint"] = -1
        chain.append(ent)
    assert len(chain) == 12 and len(jnames) == 8, (len(chain), jnames)

    # ---- collision tree in KDL DFS order
    tree = []
    index = {}

    def expand(name, parent_idx):
        for ch in children.get(name, []):
            j = by_child[ch]
            ent = {"name": ch, "parent": parent_idx}
            if ch in PLAN_JOINT_LINKS:
                ent["joint"] = PLAN_JOINT_LINKS.index(ch)
                ent["type"] = j.kdl_type
                ent["axis"] = j.axis
                ent["origin"] = j.F[1]
                ent["R"] = list(IDENT[0])
                ent["p"] = [0.0, 0.0, 0.0]
            else:
                ent["joint"] = -1
                ent["type"] = "None"
                ent["axis"] = [0.0, 0.0, 0.0]
                ent["origin"] = [0.0, 0.0, 0.0]
                R, p = j.frame_to_tip()
                ent["R"], ent["p"] = R, p
            tree.append(ent)
            index[ch] = len(tree) - 1
            expand(ch, len(tree) - 1)

    tree.append({"name": "base_link_origin", "parent": -1, "joint": -1, "type": "None",
                 "axis": [0.0, 0.0, 0.0], "origin": [0.0, 0.0, 0.0], "R": list(IDENT[0]), "p": [0.0, 0.0, 0.0]})
    index["base_link_origin"] = 0
    expand("base_link_origin", 0)
    assert len(tree) == 39

    # collision geometry + the transformToParent *= frameAdjust quirk (applied to movable links too,
    # where it is ignored because updateTransforms uses joint->pose for them)
    geom = {}
    for name, el in links.items():
        c = el.find("collision")
        if c is None:
            continue
        g = c.find("geometry")[0]
        o = c.find("origin")
        xyz = parse_floats(o.get("xyz") if o is not None else None)
        rpy = parse_floats(o.get("rpy") if o is not None else None)
        ok = True
        if g.tag == "box":
            dims = parse_floats(g.get("size"))
            ok = all(d > 0 for d in dims)
            geom[name] = ("box", dims)
        elif g.tag == "cylinder":
            geom[name] = ("cylinder", [float(g.get("radius")), float(g.get("length"))])
        elif g.tag == "sphere":
            geom[name] = ("sphere", [float(g.get("radius"))])
        else:
            geom[name] = ("mesh", [g.get("filename")])
        if not ok:
            del geom[name]
            continue
        adj = (rot_from_quat(*quat_from_rpy(*rpy)), xyz)
        e = tree[index[name]]
        if e["joint"] < 0:
            e["R"], e["p"] = frame_mul((e["R"], e["p"]), adj)
        e["collision"] = True
    for e in tree:
        e.setdefault("collision", False)

    # ---- collision geometry per link (collision-frame coordinates, the frame FCL places the object in):
    # URDF box / cylinder primitives stay exact (prims, below); mesh links get sphere covers (SPHERE_SPEC)
    spec = sphere_spec()
    for link in spec:
        if link not in index or not tree[index[link]].get("collision"):
            raise SystemExit("sphere spec names a link without collision geometry: " + link)
    S = []
    for i, e in enumerate(tree):  # tree order, spheres in spec order (the C++ builder reads them the same way)
        for x, y, z, r in spec.get(e["name"], []):
            S.append({"link": i, "c": [float(x), float(y), float(z)], "r": float(r)})

    coll_links = [i for i, e in enumerate(tree) if e["collision"]]
    prim_links = [i for i in coll_links if geom[tree[i]["name"]][0] in ("box", "cylinder") and tree[i]["name"] not in spec]
    for i in coll_links:
        assert i in prim_links or any(s["link"] == i for s in S), "no geometry for " + tree[i]["name"]

    # ---- self pairs (SRDF disabled pairs removed)
    dis = set()
    for d in srdf.findall("disable_collisions"):
        dis.add(frozenset((d.get("link1"), d.get("link2"))))
    pairs = [[a, b] for a, b in itertools.combinations(coll_links, 2)
             if frozenset((tree[a]["name"], tree[b]["name"])) not in dis]
    assert len(pairs) == 230, len(pairs)
    # A pair whose relative pose depends on no planning joint is rigid: its collision state is the same for
    # every q.  The reference re-tests it on every call (collision_checker.hpp:541-552) and, for a robot
    # that can move at all, always finds it free; it is therefore evaluated once here (as free) and dropped.
    def joint_set(i):
        js = set()
        while i >= 0:
            if tree[i]["joint"] >= 0:
                js.add(tree[i]["joint"])
            i = tree[i]["parent"]
        return js
    rigid = [p for p in pairs if not (joint_set(p[0]) ^ joint_set(p[1]))]
    pairs = [p for p in pairs if p not in rigid]

    # ---- rigid-body collapse: every link hangs rigidly off its nearest movable ancestor-or-self
    # ("body").  The chain of frame products to the bodies is kept exactly as the tree recursion
    # (CC:519-539); sphere centres / primitive frames / link bounds are pre-composed into their body frame.
    def body_of(i):
        while tree[i]["joint"] < 0:
            i = tree[i]["parent"]
        return i

    def offset(body, i):  # F_{body+1} * ... * F_i, left-associated like the tree recursion
        path = []
        while i != body:
            path.append(i)
            i = tree[i]["parent"]
        f = (list(IDENT[0]), [0.0, 0.0, 0.0])
        first = True
        for k in reversed(path):
            fk = (tree[k]["R"], tree[k]["p"])
            f = fk if first else frame_mul(f, fk)
            first = False
        return f, first

    def to_body(b, i, c):  # point c of link i's collision frame in body b's frame
        (R, pp), ident = offset(b, i)
        if ident:
            return list(c)
        m = rot_vec(R, c)
        return [m[d] + pp[d] for d in range(3)]

    bodies = sorted({body_of(s["link"]) for s in S} | {body_of(i) for i in prim_links})
    body_chain = []
    for k in range(1, max(bodies) + 1):
        e = tree[k]
        assert e["parent"] == k - 1, "body chain must be a path"
        body_chain.append({"link": k, "type": e["type"], "joint": e["joint"], "axis": e["axis"],
                           "origin": e["origin"], "R": e["R"], "p": e["p"],
                           "body": bodies.index(k) if k in bodies else -1})

    # A body is planar when every step of its chain keeps the world z axis: prismatic axes in the xy plane,
    # revolute axes along +-z, fixed frames rotating about z only.  Its world frame is then Trans(x, y, z0) Rz(a) with
    # a constant z0, and a primitive whose own z axis is vertical in it stays an upright box / cylinder.
    def planar(b):
        for k in range(1, b + 1):
            e = tree[k]
            if e["joint"] >= 0:
                ax = e["axis"]
                if e["type"] == "TransAxis" and ax[2] != 0.0:
                    return False
                if e["type"] == "RotAxis" and not (ax[0] == 0.0 and ax[1] == 0.0 and abs(ax[2]) == 1.0):
                    return False
            else:
                R = e["R"]
                if not (R[2] == 0.0 and R[5] == 0.0 and R[6] == 0.0 and R[7] == 0.0 and R[8] == 1.0):
                    return False
        return True

    for sp in S:
        b = body_of(sp["link"])
        sp["body"] = bodies.index(b)
        sp["cb"] = to_body(b, sp["link"], sp["c"])
    prims = []
    for i in prim_links:
        b = body_of(i)
        kind, dims = geom[tree[i]["name"]]
        (R, pp), ident = offset(b, i)
        if not planar(b):
            raise SystemExit("primitive on a non-planar body (give it spheres in the sphere spec): " + tree[i]["name"])
        # the primitive's z axis in the body frame (column 2 of the offset rotation) must be vertical up to rounding
        # (kinect_link: rpy 1.57 then -1.57 about x, a residual tilt of 1e-16 rad); it is then taken as vertical
        if abs(R[2]) > 1e-9 or abs(R[5]) > 1e-9 or abs(R[8] - 1.0) > 1e-9 or abs(R[6]) > 1e-9:
            raise SystemExit("primitive not upright in its planar body: " + tree[i]["name"])
        if kind == "box":
            half = [0.5 * dims[0], 0.5 * dims[1], 0.5 * dims[2]]
            rxy = math.sqrt(half[0] * half[0] + half[1] * half[1])
            rall = math.sqrt(half[0] * half[0] + half[1] * half[1] + half[2] * half[2])
        else:
            half = [dims[0], 0.5 * dims[1], 0.0]
            rxy = dims[0]
            rall = math.sqrt(half[0] * half[0] + half[1] * half[1])
        prims.append({"link": i, "body": bodies.index(b), "type": kind, "half": half,
                      "cb": list(pp) if not ident else [0.0, 0.0, 0.0],
                      "ab": [R[0], R[3], 0.0] if not ident else [1.0, 0.0, 0.0],
                      "rxy": rxy + 1e-6, "r": rall + 1e-6})
    # per-link bounding spheres (prefilter for the self-collision pair test), margin 1e-6; sums in list order
    lbs = []
    for i in coll_links:
        b = body_of(i)
        pr = [q for q in prims if q["link"] == i]
        if pr:
            cb, r = list(pr[0]["cb"]), pr[0]["r"]
            c = [0.0, 0.0, 0.0]
        else:
            ss = [q for q in S if q["link"] == i]
            c = [0.0, 0.0, 0.0]
            for q in ss:
                c = [c[d] + q["c"][d] for d in range(3)]
            c = [c[d] / len(ss) for d in range(3)]
            r = 0.0
            for q in ss:
                dx, dy, dz = q["c"][0] - c[0], q["c"][1] - c[1], q["c"][2] - c[2]
                r = max(r, math.sqrt(dx * dx + dy * dy + dz * dz) + q["r"])
            r = r + 1e-6
            cb = to_body(b, i, c)
        lbs.append({"link": i, "c": c, "r": r, "body": bodies.index(b), "cb": cb})

    model = {
        "format": "smp-robot-model-2",
        "source": "tpatten/squirrel_motion_planner squirrel_8dof_planner/config/robotino_plan.{urdf,srdf}, "
                  "squirrel-hand.dae; sphere covers in squirrel_motion_planner_amd/data/robotino_spheres.json",
        "root_z": 0.02, "octree_z_offset": -0.02,
        "joint_names": jnames, "q_min": qmin, "q_max": qmax, "joint_is_revolute": jrev,
        "chain": chain, "links": tree,
        "spheres": S,
        "prims": prims,
        "link_bounds": lbs,
        "bodies": bodies,
        "body_chain": body_chain,
        "self_pairs": pairs,
        "self_pairs_srdf_enabled": 230,
        "self_pairs_rigid_dropped": [[tree[a]["name"], tree[b]["name"]] for a, b in rigid],
    }
    return model


def main():
    model = build_model()
    validate(model, REF)
    with open(OUT, "w") as f:
        json.dump(model, f, indent=1)
    spec = {"format": "smp-sphere-spec-1",
            "about": "sphere covers of the mesh collision links in each link's collision frame, [x, y, z, r] in m "
                     "(tools/gen_robot_model.py); box / cylinder links of the URDF are collided exactly",
            "links": {model["links"][i]["name"]: v for i, v in
                      sorted((tree_index, v) for tree_index, v in
                             ((next(k for k, e in enumerate(model["links"]) if e["name"] == n), v)
                              for n, v in sphere_spec().items()))}}
    with open(SPEC_OUT, "w") as f:
        json.dump(spec, f, indent=1)
    print("wrote", OUT, len(model["spheres"]), "spheres", len(model["self_pairs"]), "pairs")


def link_frames(model, q):
    T = []
    for e in model["links"]:
        if e["parent"] < 0:
            T.append((list(IDENT[0]), [0.0, 0.0, model["root_z"]]))
            continue
        P = T[e["parent"]]
        if e["joint"] >= 0:
            if e["type"] == "RotAxis":
                L = (rot2(e["axis"], q[e["joint"]]), e["origin"])
            else:
                L = (list(IDENT[0]), [e["origin"][i] + e["axis"][i] * q[e["joint"]] for i in range(3)])
        else:
            L = (e["R"], e["p"])
        T.append(frame_mul(P, L))
    return T


def prim_world(model, T, pr):
    R, p = T[model["bodies"][pr["body"]]]
    c = rot_vec(R, pr["cb"])
    u = rot_vec(R, pr["ab"])
    return [c[i] + p[i] for i in range(3)], u


def sphere_prim_gap(w, pr, cw, u):
    """Distance from point w to an upright box / cylinder (0 inside) -- the generator's check, not the parity path."""
    dx, dy, dz = w[0] - cw[0], w[1] - cw[1], w[2] - cw[2]
    h = pr["half"]
    if pr["type"] == "box":
        lx, ly = u[0] * dx + u[1] * dy, -u[1] * dx + u[0] * dy
        qx, qy, qz = max(abs(lx) - h[0], 0.0), max(abs(ly) - h[1], 0.0), max(abs(dz) - h[2], 0.0)
    else:
        qx, qy, qz = max(math.hypot(dx, dy) - h[0], 0.0), 0.0, max(abs(dz) - h[1], 0.0)
    return math.sqrt(qx * qx + qy * qy + qz * qz)


def self_collisions(model, q):
    T = link_frames(model, q)
    W = {}
    for s in model["spheres"]:
        R, p = T[model["bodies"][s["body"]]]
        c = rot_vec(R, s["cb"])
        W.setdefault(s["link"], []).append(([c[i] + p[i] for i in range(3)], s["r"]))
    P = {pr["link"]: (pr,) + tuple(prim_world(model, T, pr)) for pr in model["prims"]}
    hits = []
    for a, b in model["self_pairs"]:
        if a in P and b in P:
            raise SystemExit("primitive-primitive pair that is not rigid")
        if a in P or b in P:
            pl, sl = (a, b) if a in P else (b, a)
            pr, cw, u = P[pl]
            best = min(sphere_prim_gap(c, pr, cw, u) - r for c, r in W[sl])
        else:
            best = min(math.dist(ca, cb) - ra - rb for ca, ra in W[a] for cb, rb in W[b])
        if best <= 0:
            hits.append((model["links"][a]["name"], model["links"][b]["name"], best))
    return hits


def mesh_evidence(model, q, link, prim_link):
    """Vertices of `link`'s kclhand mesh (squirrel-hand.dae) inside the exact primitive of prim_link at q."""
    import hand_spheres
    meshes, _ = hand_spheres.load_dae(os.path.join(REF, "squirrel-hand.dae"))
    if link not in meshes:
        return None
    names = [e["name"] for e in model["links"]]
    T = link_frames(model, q)
    R, p = T[names.index(link)]
    V = meshes[link].reshape(-1, 3)
    W = [[sum(R[r * 3 + k] * v[k] for k in range(3)) + p[r] for r in range(3)] for v in V[::3]]
    pr = [x for x in model["prims"] if model["links"][x["link"]]["name"] == prim_link][0]
    cw, u = prim_world(model, T, pr)
    return sum(1 for w in W if sphere_prim_gap(w, pr, cw, u) == 0.0), len(W)


def validate(model, ref):
    import re
    txt = open(os.path.join(ref, "parameters.yaml")).read()
    folded = [float(v) for v in re.search(r"pose_folded_arm:\s*\[([^\]]*)\]", txt).group(1).split(",")]
    keys = [("pose_folded_arm", 0, folded)]
    for fn in ("folding_poses_tuw-robotino2.yaml", "folding_poses_uibk-robotino2.yaml", "folding_poses_alufr-robotino.yaml"):
        t2 = open(os.path.join(ref, fn)).read()
        traj = [float(v) for v in re.search(r"trajectory_folding_arm:\s*\[([^\]]*)\]", t2, re.S).group(1).split(",")]
        keys += [(fn, i // 5, traj[i:i + 5]) for i in range(0, len(traj), 5)]
    report = []
    prim_names = {model["links"][p["link"]]["name"] for p in model["prims"]}
    for fn, i, k in keys:
        hits = self_collisions(model, [0.0, 0.0, 0.0] + k)
        for a, b, gap in hits:
            ev = None
            if a in prim_names or b in prim_names:
                pl, ml = (a, b) if a in prim_names else (b, a)
                ev = mesh_evidence(model, [0.0, 0.0, 0.0] + k, ml, pl)
            report.append((fn, i, a, b, gap, ev))
            print("keyframe %s[%d] self-collides: %s / %s (sphere gap %.4f m)%s" %
                  (fn, i, a, b, gap, "" if ev is None else
                   "; exact primitive vs the link's mesh: %d of %d sampled vertices inside" % ev), file=sys.stderr)
    # A keyframe may only be in collision if one of its colliding pairs is a hand mesh (squirrel-hand.dae) entering an
    # exact URDF primitive: then the reference's FCL check finds that keyframe in collision too.  Further pairs of such
    # a keyframe may be sphere-cover overshoot (the cover is conservative).
    for fn, i in sorted({(r[0], r[1]) for r in report}):
        if not any(r[5] is not None and r[5][0] > 0 for r in report if (r[0], r[1]) == (fn, i)):
            raise SystemExit("model invalid: keyframe %s[%d] collides without a mesh-level cause" % (fn, i))
    return report


if __name__ == "__main__":
    main()
