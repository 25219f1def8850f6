#!/usr/bin/env python3
"""Sphere covers of the kclhand collision meshes (offline; reads the reference's squirrel-hand.dae).

The reference collides the hand links as FCL OBBRSS meshes (collision_checker.hpp:301) loaded from
package://robotino_description/meshes/kclhand/*.STL (robotino_plan.urdf:897-1180).  That package is absent, but
squirrel_8dof_planner/config/squirrel-hand.dae holds the same 11 meshes as a COLLADA scene: one node per link, named
after the link, whose matrix is the URDF joint origin (hand_base_link: rpy 0 0.52 0 at (-0.02105, 0.1485, 0),
robotino_plan.urdf:877-879), so each geometry's positions are in its link frame.

A cover here is a set of spheres such that every mesh triangle lies inside one of them (a ball is convex, so a
sphere holding a triangle's three vertices holds the triangle): every configuration where the mesh touches a voxel
or another link is also one where a sphere does -- the sphere model is conservative, never optimistic.
Fitting: k-means on triangle centroids (deterministic init), then per cluster the minimum enclosing ball of its
triangles' vertices (Welzl's exact algorithm in 3-D on the cluster's vertices), a few rounds of reassigning each
triangle to the sphere whose radius grows least.
"""
import os
import xml.etree.ElementTree as ET

import numpy as np

NS = {"c": "http://www.collada.org/2005/11/COLLADASchema"}


def load_dae(path):
    """{link name: triangles (n, 3, 3) in the link frame} and {link name: node matrix (4, 4)}."""
    root = ET.parse(path).getroot()
    geoms = {}
    for g in root.iter("{%s}geometry" % NS["c"]):
        mesh = g.find("c:mesh", NS)
        pos = None
        for src in mesh.findall("c:source", NS):
            if src.get("id").endswith("positions"):
                pos = np.array(src.find("c:float_array", NS).text.split(), float).reshape(-1, 3)
        tris = []
        for pl in mesh.findall("c:polylist", NS):
            inputs = pl.findall("c:input", NS)
            stride = max(int(i.get("offset")) for i in inputs) + 1
            voff = [int(i.get("offset")) for i in inputs if i.get("semantic") == "VERTEX"][0]
            vc = np.array(pl.find("c:vcount", NS).text.split(), int)
            p = np.array(pl.find("c:p", NS).text.split(), int).reshape(-1, stride)[:, voff]
            if not np.all(vc == 3):
                raise ValueError("non-triangle polygons in " + g.get("id"))
            tris.append(pos[p].reshape(-1, 3, 3))
        geoms["#" + g.get("id")] = np.concatenate(tris)
    out, mats = {}, {}

    def walk(n):
        for ch in n.findall("c:node", NS):
            ig = ch.find("c:instance_geometry", NS)
            if ig is not None:
                out[ch.get("name")] = geoms[ig.get("url")]
                mats[ch.get("name")] = np.array(ch.find("c:matrix", NS).text.split(), float).reshape(4, 4)
            walk(ch)

    walk(root.find("c:library_visual_scenes", NS).find("c:visual_scene", NS))
    return out, mats


def min_ball(P):
    """Exact minimum enclosing ball of points P (m, 3): Welzl's algorithm (move-to-front, iterative over a shuffled
    copy with a fixed seed).  Returns (centre, radius)."""
    P = np.unique(np.round(P, 12), axis=0)
    rng = np.random.default_rng(0)
    P = P[rng.permutation(len(P))]

    def ball_of(R):
        if len(R) == 0:
            return np.zeros(3), -1.0
        if len(R) == 1:
            return R[0].copy(), 0.0
        A = np.array(R)
        # circumsphere of up to 4 points in their affine hull: c = A0 + sum t_i (Ai - A0), |c - Ai| equal
        B = A[1:] - A[0]
        M = B @ B.T
        rhs = 0.5 * np.einsum("ij,ij->i", B, B)
        t = np.linalg.lstsq(M, rhs, rcond=None)[0]
        c = A[0] + t @ B
        return c, float(np.max(np.linalg.norm(A - c, axis=1)))

    def inside(c, r, p):
        return r >= 0 and np.linalg.norm(p - c) <= r * (1 + 1e-12) + 1e-15

    def mb(pts, R):
        c, r = ball_of(R)
        if len(R) == 4:
            return c, r
        for i in range(len(pts)):
            if not inside(c, r, pts[i]):
                c, r = mb(pts[:i], R + [pts[i]])
        return c, r

    import sys
    sys.setrecursionlimit(10000)
    # iterative outer loop (the recursion depth is bounded by the support size, 4)
    c, r = ball_of([])
    for i in range(len(P)):
        if not inside(c, r, P[i]):
            c, r = mb(P[:i], [P[i]])
    return c, r


def subdivide(tris, max_edge):
    """Split triangles at the midpoint of their longest edge until no edge exceeds max_edge (the pieces tile the
    original triangles, so covering every piece covers the mesh)."""
    out = []
    todo = tris
    while len(todo):
        e = np.stack([np.linalg.norm(todo[:, 1] - todo[:, 0], axis=1), np.linalg.norm(todo[:, 2] - todo[:, 1], axis=1),
                      np.linalg.norm(todo[:, 0] - todo[:, 2], axis=1)], 1)
        done = e.max(1) <= max_edge
        out.append(todo[done])
        T = todo[~done]
        if not len(T):
            break
        k = e[~done].argmax(1)  # longest edge k: vertices (k, k+1)
        a = T[np.arange(len(T)), k]
        b = T[np.arange(len(T)), (k + 1) % 3]
        c = T[np.arange(len(T)), (k + 2) % 3]
        m = 0.5 * (a + b)
        todo = np.concatenate([np.stack([a, m, c], 1), np.stack([m, b, c], 1)])
    return np.concatenate(out)


def fit(tris, k, rounds=4):
    """k spheres covering every triangle of tris (n, 3, 3)."""
    tris = subdivide(tris, MAX_EDGE)
    cen = tris.mean(1)
    # deterministic farthest-point init from the centroid of all
    idx = [int(np.argmax(np.linalg.norm(cen - cen.mean(0), axis=1)))]
    for _ in range(1, k):
        d = np.min(np.linalg.norm(cen[:, None] - cen[idx][None], axis=2), axis=1)
        idx.append(int(np.argmax(d)))
    C = cen[idx].copy()
    for _ in range(30):
        lab = np.argmin(np.linalg.norm(cen[:, None] - C[None], axis=2), axis=1)
        C = np.array([cen[lab == j].mean(0) if np.any(lab == j) else C[j] for j in range(k)])
    balls = None
    for _ in range(rounds):
        balls = []
        for j in range(k):
            T = tris[lab == j]
            if len(T) == 0:
                balls.append((C[j], 0.0))
                continue
            balls.append(min_ball(T.reshape(-1, 3)))
        # reassign each triangle to the ball whose radius it enlarges least (0 if it fits already)
        need = np.stack([np.max(np.linalg.norm(tris - c[None, None], axis=2), axis=1) - r for c, r in balls], 1)
        lab = np.argmin(np.maximum(need, 0.0) + 1e-9 * np.linalg.norm(cen[:, None] - np.array([b[0] for b in balls])[None], axis=2), axis=1)
    balls = [min_ball(tris[lab == j].reshape(-1, 3)) for j in range(k) if np.any(lab == j)]
    # every triangle inside some ball (exact check, tiny tolerance for the enclosing-ball solve)
    V = tris.reshape(-1, 3, 3)
    ok = np.zeros(len(V), bool)
    for c, r in balls:
        ok |= np.all(np.linalg.norm(V - c[None, None], axis=2) <= r + 1e-9, axis=1)
    assert ok.all(), "cover failed"
    return balls


# spheres per link: the fingers are 66 / 56 mm long rods of ~16 mm, the couplers and cranks short bars, the hand base
# a block of 65 x 126 x 87 mm
K = {"hand_base_link": 8,
     "hand_left_crank": 1, "hand_right_crank": 1, "hand_left_coupler": 2, "hand_right_coupler": 2,
     "hand_left_finger_lower_link": 3, "hand_middle_finger_lower_link": 3, "hand_right_finger_lower_link": 3,
     "hand_left_finger_upper_link": 3, "hand_middle_finger_upper_link": 3, "hand_right_finger_upper_link": 3}

MAX_EDGE = 0.004  # triangles are split to 4 mm pieces before clustering (a long sliver would force one large ball)
MARGIN = 1e-4  # 0.1 mm on top of the exact cover: rounding of the stored centres and radii


def hand_spheres(dae_path):
    """{link: [[x, y, z, r], ...]} in the link frame, plus a report {link: (n triangles, max radius)}."""
    meshes, _ = load_dae(dae_path)
    out, rep = {}, {}
    for link, k in K.items():
        balls = fit(meshes[link], k)
        out[link] = [[round(float(c[0]), 6), round(float(c[1]), 6), round(float(c[2]), 6),
                      round(float(r) + MARGIN + 2e-6, 6)] for c, r in balls]
        rep[link] = (len(meshes[link]), max(r for c, r in balls))
    return out, rep


if __name__ == "__main__":
    import json
    import sys
    s, rep = hand_spheres(sys.argv[1] if len(sys.argv) > 1 else
                          "/root/reference/squirrel_8dof_planner/config/squirrel-hand.dae")
    for k, v in rep.items():
        print("%-32s %6d triangles  %d spheres  max r %.4f" % (k, v[0], len(s[k]), v[1]))
    print(json.dumps(s))
