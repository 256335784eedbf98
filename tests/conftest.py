import os
import sys

import pytest

try:  # first, so that librtw.so binds to the HIP runtime torch ships (one runtime per process)
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def assets():
    from raytracinginaweekend_amd.assets import load_assets

    return load_assets()


@pytest.fixture(scope="session")
def worlds(assets):
    import raytracinginaweekend_amd as R

    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = R.demo_world(name, assets)
        return cache[name]

    return get
