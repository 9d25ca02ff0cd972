"""Shared fixtures.  `-m "not gpu"` runs on CPU only (compiler, oracle, host logic, ABI symbols);
`-m gpu` tests call the HIP path through the C ABI and compare with the fp64 oracle."""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

REF_SCENE = ROOT / "tests" / "golden" / "ref_scenes" / "scene.xml"
REF_PID_SCENE = ROOT / "tests" / "golden" / "ref_scenes" / "test_pid" / "scene_pid.xml"
ARM7 = ROOT / "scenes" / "arm7_lidar.xml"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session", autouse=True)
def built():
    from mujoco_ros2_simulation_amd import build
    build.build_lib()
    build.build_plugin()
    build.build_oracle()
    # torch's own HIP runtime initialises first: a test that reaches torch.cuda only after the library
    # has driven the GPU (a subset run starting with such tests) otherwise sees "No HIP GPUs are
    # available" on the box
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    return True


@pytest.fixture(scope="session")
def s2_model(built):
    from mujoco_ros2_simulation_amd import sim
    return sim.Model.load(REF_SCENE)


@pytest.fixture(scope="session")
def pid_model(built):
    from mujoco_ros2_simulation_amd import sim
    return sim.Model.load(REF_PID_SCENE)


@pytest.fixture(scope="session")
def arm7_model(built):
    from mujoco_ros2_simulation_amd import sim
    return sim.Model.load(ARM7)


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
