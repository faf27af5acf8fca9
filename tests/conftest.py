import os
import sys

import pytest
# torch before the engine: the ROCm wheel of torch brings its own HIP runtime, and libskirt_amd.so then binds
# to that same runtime (one libamdhip64.so.7 per process); loaded the other way round, torch finds no GPU in a
# process whose engine already initialized the system runtime (test_dust_labs_bound_after_a_stellar_phase)
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")
