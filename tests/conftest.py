import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REF_CONFIG = "/root/reference/squirrel_8dof_planner/config"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: longer CPU-oracle runs")


def have_reference():
    return os.path.isdir(REF_CONFIG)


@pytest.fixture(scope="session")
def model_path():
    return os.path.join(ROOT, "squirrel_motion_planner_amd", "data", "robotino_model.json")


@pytest.fixture(scope="session")
def orobot(model_path):
    from oracle import oracle as O
    return O.OracleRobot(model_path)
