import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "sift-features_amd"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path")
    config.addinivalue_line("markers", "slow: long-running full-size case")


@pytest.fixture(scope="session")
def pkg():
    import pkg_loader
    return pkg_loader.load()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def ctx(pkg):
    c = pkg.Context(0, pkg.OpenCVProcessing)
    yield c
    c.close()


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    return {k: d[k] for k in d.files}


@pytest.fixture(scope="session")
def synth():
    import synth as S
    return S
