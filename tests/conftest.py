import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "open3d-py-extension_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and libo3dx.so")
    config.addinivalue_line("markers", "slow: large-size property tests")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def dev():
    import torch

    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def bunny():
    from open3dpypro.pcd_io import read_pcd_arrays

    fields = read_pcd_arrays(os.path.join(GOLDEN, "bunny.pcd"))
    import numpy as np

    return np.stack([fields["x"], fields["y"], fields["z"]], 1).astype(np.float32)
