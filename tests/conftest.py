import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))  # test infrastructure: the checker
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def golden(name):
    import numpy as np

    return np.load(os.path.join(GOLDEN, name + ".npz"))


def rel_err(got, ref):
    """||got - ref|| / ||ref|| in fp64 (north_star's relative bar for pose
    deltas: 1e-4)."""
    import numpy as np

    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    n = np.linalg.norm(ref)
    assert n > 0, "reference delta is zero: nothing to compare"
    return float(np.linalg.norm(got - ref) / n)


REL_TOL = 1e-4  # BASELINE.json north_star: pose deltas within 1e-4 relative


def assert_ba_rel(P, K, Pr, Kr, P0, K0, t0, t1, dX=None, dXr=None, tol=REL_TOL):
    """The product BA against the oracle at north_star's bar: the pose delta
    of the free poses, the inverse-depth delta of every patch and (when
    given) the last iteration's pose step dX, each ||got - ref|| / ||ref||
    <= tol."""
    e = {"dP": rel_err(P[t0:t1] - P0[t0:t1], Pr[t0:t1] - P0[t0:t1]),
         "dZ": rel_err(K[:, 2] - K0[:, 2], Kr[:, 2] - K0[:, 2])}
    if dX is not None:
        e["dX"] = rel_err(dX, dXr)
    assert all(v <= tol for v in e.values()), e
    return e
