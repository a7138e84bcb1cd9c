import glob
import importlib
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")
PKG_NAME = "chainer_realtime_multi-person_pose_estimation_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


def pkg_module(sub=None):
    return importlib.import_module(PKG_NAME + ("." + sub if sub else ""))


@pytest.fixture(scope="session")
def pkg():
    return pkg_module()


@pytest.fixture(scope="session")
def lib():
    return pkg_module("_lib")


@pytest.fixture(scope="session")
def rand_weights():
    return pkg_module("weights").random_weights(seed=0)


@pytest.fixture(scope="session")
def rand_weights_small():
    """Random CocoPoseNet weights scaled for the tiny precise-mode cases (same generator)."""
    return pkg_module("weights").random_weights(seed=1)


@pytest.fixture(scope="session")
def ctx(lib, rand_weights):
    c = lib.Context(0)
    c.set_weights(rand_weights)
    yield c
    c.close()


def golden_cases():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not p.endswith("gauss_scipy.npz") and not p.endswith("grouping_indexerror.npz"))


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def people_image():
    from PIL import Image
    return np.ascontiguousarray(np.asarray(Image.open(os.path.join(GOLDEN, "people.png")).convert("RGB"))[:, :, ::-1])
