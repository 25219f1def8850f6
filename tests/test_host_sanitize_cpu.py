"""ASAN / UBSAN build of the host parsers, run over truncated, bit-flipped and garbage inputs.

The octomap readers (.bt / .ot files and headerless octomap_msgs payloads, squirrel_8dof_planner.cpp:862-917), the
URDF / SRDF / sphere-spec reader (smp_urdf.cpp, the node's robot description) and the model JSON reader take bytes
from outside the process; trajectory normalisation takes caller arrays.  tests/cpp/fuzz_host.cpp drives them; a
sanitizer report aborts the harness (-fno-sanitize-recover)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle import octomap_bt

CSRC = os.path.join(ROOT, "squirrel_motion_planner_amd", "csrc")
GOLD = os.path.join(ROOT, "tests", "golden")
DATA = os.path.join(ROOT, "squirrel_motion_planner_amd", "data")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("fuzz") / "fuzz_host")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", os.path.join(ROOT, "tests", "cpp", "fuzz_host.cpp"),
           os.path.join(CSRC, "smp_host.cpp"), os.path.join(CSRC, "smp_urdf.cpp"), os.path.join(CSRC, "smp_traj.cpp"),
           "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None) if "asan" in env.get("LD_PRELOAD", "") else None
    p = subprocess.run([exe] + list(args), capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-3000:]
    ok = p.stdout.split()
    assert ok[0] == "ok"
    return int(ok[1]), int(ok[2]), int(ok[3])


def test_octomap_full_format(harness):
    n, acc, rej = run(harness, os.path.join(GOLD, "room3.ot"), "ot")
    assert acc > 0 and rej > 0


def test_octomap_binary_format(harness, tmp_path):
    keys = np.load(os.path.join(GOLD, "room4_keys.npz"))["keys"].astype(np.int64)
    bt = tmp_path / "room4.bt"
    bt.write_bytes(octomap_bt.write_bt(keys, 0.05))
    n, acc, rej = run(harness, str(bt), "bt")
    assert acc > 0 and rej > 0


def test_robot_description(harness):
    n, acc, rej = run(harness, os.path.join(GOLD, "robotino_plan.urdf"), "urdf", os.path.join(GOLD, "robotino_plan.srdf"),
                      os.path.join(DATA, "robotino_spheres.json"))
    assert acc > 0 and rej > 0


def test_model_json(harness):
    n, acc, rej = run(harness, os.path.join(DATA, "robotino_model.json"), "json")
    assert acc > 0 and rej > 0
