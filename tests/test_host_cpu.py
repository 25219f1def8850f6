"""CPU tests of the product library's host side: ABI exports, scene builder vs the oracle, .bt decoding,
and that compute entry points refuse to run without a GPU (no CPU fallback)."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from oracle import octomap_bt, oracle as O
from squirrel_motion_planner_amd import _lib as L
from squirrel_motion_planner_amd import scenes
from squirrel_motion_planner_amd.planner import Robot, Scene
from conftest import REF_CONFIG, ROOT, have_reference

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "smp_gpu.h")).read()
    return sorted(set(re.findall(r"\b(smp_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    lib = L.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert {n for n, _, _ in L.EXPORTS} == set(syms)


def test_robot_model_loads():
    r = Robot()
    names = r.link_names
    assert len(names) == 39 and names[0] == "base_link_origin" and "hand_wrist_link" in names


def _compare_scene(keys, res):
    s = Scene.from_keys(keys, res)
    o = O.OracleScene(keys, res)
    info = s.info()
    assert info["dims"] == (o.nx, o.ny, o.nz)
    assert info["origin"] == (o.ox, o.oy, o.oz)
    bits, d2 = s.export()
    assert np.array_equal(bits, o.bits)
    assert np.array_equal(d2, o.d2)


@pytest.mark.parametrize("mk", [scenes.empty_room, scenes.box_room, scenes.narrow_passage])
def test_scene_builder_matches_oracle(mk):
    sc = mk()
    _compare_scene(sc.keys, sc.res)


@pytest.mark.parametrize("room", ["room3", "room4", "room5"])
def test_room_scene_with_floor(room):
    f = np.load(os.path.join(GOLD, room + "_keys.npz"))
    keys = f["keys"].astype(np.int64)
    floor = scenes.floor_keys([0.5, -1.0], 0.05, 3.0)
    _compare_scene(np.concatenate([keys, floor]), 0.05)
    # product-side floor insertion (smp_scene_opts.insert_floor) equals the explicit keys
    a = Scene.from_keys(keys, 0.05, floor_center=(0.5, -1.0), floor_distance=3.0).export()
    b = Scene.from_keys(np.concatenate([keys, floor]), 0.05).export()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_edt_random_grids():
    rng = np.random.default_rng(5)
    for _ in range(5):
        n = rng.integers(1, 400)
        keys = 32768 + rng.integers(0, 30, (n, 3))
        _compare_scene(keys, 0.05)


def test_empty_scene():
    _compare_scene(np.zeros((0, 3)), 0.05)


@pytest.mark.parametrize("room", ["room3", "room4", "room5"])
def test_bt_decoder(room):
    f = np.load(os.path.join(GOLD, room + "_keys.npz"))
    keys = f["keys"].astype(np.int64)
    data = octomap_bt.write_bt(keys, 0.05)
    a = Scene.from_bt(data).export()
    b = Scene.from_keys(keys, 0.05).export()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    if have_reference():  # the reference's own (pruned) file
        raw = open(os.path.join(REF_CONFIG, room + ".bt"), "rb").read()
        c = Scene.from_bt(raw).export()
        assert np.array_equal(c[0], b[0]) and np.array_equal(c[1], b[1])


def test_bt_parse_errors():
    with pytest.raises(L.SmpError):
        Scene.from_bt(b"# Octomap OcTree binary file\nid OcTree\nsize 3\nres 0.05\ndata\n\x03")


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = Robot()
    h = ctypes.c_void_p()
    p = L.Params()
    L.lib().smp_params_default(ctypes.byref(p))
    st = L.lib().smp_planner_create(0, r.h, ctypes.byref(p), ctypes.byref(h))
    assert st == L.SMP_ERR_NO_DEVICE


GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _description():
    return (open(os.path.join(GOLD, "robotino_plan.urdf")).read(), open(os.path.join(GOLD, "robotino_plan.srdf")).read())


def test_urdf_path_builds_the_committed_model():
    """smp_robot_create_urdf (C++ XML reader, KDL segment rules, float-cast limits, SRDF pairs, exact primitives, body
    collapse) gives the device model of the committed JSON (tools/gen_robot_model.py, Python) byte for byte."""
    urdf, srdf = _description()
    a = Robot().device_bytes()
    b = Robot.from_urdf(urdf, srdf).device_bytes()
    assert len(a) == len(b) and a == b
    assert Robot.from_urdf(urdf, srdf).link_names == Robot().link_names


def test_urdf_path_errors():
    urdf, srdf = _description()
    bad = [(urdf[: len(urdf) // 2], srdf), ("<robot><link name='a'/></robot>", srdf), (urdf, "<robot/>"),
           ("not xml", srdf), (urdf.replace('<box size="0.55 0.55 0.17"/>', '<box size="0.55 0.55"/>'), srdf)]
    for u, s in bad:
        h = ctypes.c_void_p()
        assert L.lib().smp_robot_create_urdf(u.encode(), s.encode(), open(L.SPHERES_JSON, "rb").read(),
                                             ctypes.byref(h)) == L.SMP_ERR_PARSE
    h = ctypes.c_void_p()
    spec = json.load(open(L.SPHERES_JSON))
    spec["links"]["no_such_link"] = [[0, 0, 0, 0.1]]
    assert L.lib().smp_robot_create_urdf(urdf.encode(), srdf.encode(), json.dumps(spec).encode(),
                                         ctypes.byref(h)) == L.SMP_ERR_PARSE
    # descriptions the model cannot place are parse errors, never out-of-bounds reads: collision geometry on the root
    # link (no planning joint above it), a joint axis of zero length, no collision link at all
    m = re.search(r'<link name="base_link_origin"\s*/?>', urdf)
    col = '<link name="base_link_origin"><collision><geometry><box size="0.1 0.1 0.1"/></geometry></collision>'
    root_box = urdf.replace(m.group(0), col + ("</link>" if m.group(0).endswith("/>") else ""))
    zero_axis = urdf.replace('<axis xyz="0 0 1"', '<axis xyz="0 0 0"', 1)
    no_col = re.sub(r"<collision>.*?</collision>", "", urdf, flags=re.S)
    spec0 = json.load(open(L.SPHERES_JSON))
    spec0["links"] = {}
    for u, sp in [(root_box, open(L.SPHERES_JSON).read()), (zero_axis, open(L.SPHERES_JSON).read()),
                  (no_col, json.dumps(spec0))]:
        assert L.lib().smp_robot_create_urdf(u.encode(), srdf.encode(), sp.encode(), ctypes.byref(h)) == L.SMP_ERR_PARSE
    # a box link given spheres in the spec is collided with those spheres instead of exactly
    spec = json.load(open(L.SPHERES_JSON))
    spec["links"]["kinect_link"] = [[0.0, 0.0, 0.0, 0.1]]
    r = Robot.from_urdf(urdf, srdf, json.dumps(spec))
    assert r.device_bytes() != Robot().device_bytes()


@pytest.mark.parametrize("mk", [scenes.box_room, scenes.clutter_cloud])
def test_primitive_slabs_match_oracle(mk, orobot):
    """The per-primitive slab prefilter fields (C++ builder) equal the oracle's independent scipy construction."""
    sc = mk()
    s = Scene.from_keys(sc.keys, sc.res)
    r = Robot()
    n = L.lib().smp_probe_scene_slabs(r.h, s.h, None, 0)
    got = np.zeros(n, np.uint16)
    L.lib().smp_probe_scene_slabs(r.h, s.h, got.ctypes.data_as(ctypes.c_void_p), n)
    orc = O.Oracle(orobot, O.OracleScene(sc.keys, sc.res))
    want = orc.scene._slab
    assert np.array_equal(got, want)
    assert orobot.n_prim == 6 and (got < 65535).any()


def test_rigid_pairs_are_configuration_independent():
    """The SRDF-enabled pairs the model leaves out (smp_get_collisions, smp_gpu.h) are pairs of links on one rigid
    body: their relative pose, and so their overlap, is the same in every configuration.  Under the sphere covers
    exactly the 7 listed in smp_gpu.h overlap (cover artefacts of touching hand parts and of door / shell)."""
    m = json.load(open(os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")))
    names = [e["name"] for e in m["links"]]
    body = {e["link"]: e["body"] for e in m["link_bounds"]}
    rigid = m["self_pairs_rigid_dropped"]
    assert len(rigid) == 65 and m["self_pairs_srdf_enabled"] == len(rigid) + len(m["self_pairs"])
    over = []
    for a, b in rigid:
        ia, ib = names.index(a), names.index(b)
        assert body[ia] == body[ib], (a, b)
        sa = [s for s in m["spheres"] if s["link"] == ia]
        sb = [s for s in m["spheres"] if s["link"] == ib]
        if sa and sb and min(np.linalg.norm(np.subtract(x["cb"], y["cb"])) - x["r"] - y["r"] for x in sa for y in sb) <= 0:
            over.append((a, b))
    assert sorted(over) == sorted([
        ("hand_base_link", "hand_left_coupler"), ("hand_base_link", "hand_left_finger_lower_link"),
        ("hand_base_link", "hand_right_coupler"), ("hand_left_crank", "hand_left_finger_lower_link"),
        ("hand_left_coupler", "hand_right_coupler"), ("hand_right_crank", "hand_right_finger_lower_link"),
        ("door_link", "shell_base_link")])
