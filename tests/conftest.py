import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def pkg():
    return importlib.import_module("loam_velodyne-1_amd")


def synth():
    return importlib.import_module("loam_velodyne-1_amd.synthgen")


@pytest.fixture(scope="session")
def loam():
    return pkg()


@pytest.fixture(scope="session")
def sg():
    return synth()


@pytest.fixture(scope="session")
def oc():
    import oracle_ctypes
    return oracle_ctypes
