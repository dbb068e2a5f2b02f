import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def built():
    """libgsplat.so + oracle are built in-tree (no-op when up to date)."""
    from gaussian_splat_amd import build
    if not build.LIB.exists() or os.environ.get("GSPLAT_REBUILD"):
        build.build_lib()
    if not (ROOT / "oracle" / "liboracle.so").exists():
        build.build_oracle()
    return True


@pytest.fixture(scope="session")
def default_cam_256():
    from gaussian_splat_amd.api import default_camera
    cam = default_camera(256, 256)
    return cam.getViewMatrix(), cam.getProjectionMatrix()


def orbit_views(width, height, n=3):
    """Reference default camera plus orbit poses."""
    from gaussian_splat_amd.api import default_camera
    out = []
    for k in range(n):
        cam = default_camera(width, height)
        if k:
            cam.orbit(0.35 * k, 0.1 * k)
        out.append((cam.getViewMatrix(), cam.getProjectionMatrix()))
    return out
