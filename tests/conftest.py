import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "real-time-ray-tracing_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def rtx():
    import rtx as R
    R.load_library()
    return R


@pytest.fixture(scope="session")
def default_scene(oracle):
    v, i, n = oracle.scene(1)
    nrm = oracle.smooth_normals(v, i)
    bvh = oracle.build_bvh(v, i, n, nrm)
    return dict(vertices=v, indices=i, tri_count=n, normals=nrm, bvh=bvh)
