"""cuda_ba.solve_system (Sim3 pose-graph solve, dpvo/fastba/ba.cpp:120-180).

CPU: the numpy oracle against an independent scipy.sparse formulation that
follows ba.cpp literally (triplets -> J, Jt*J, diagonal damping, solve of the
top-left block).  Parity unpinned otherwise: the reference needs Eigen, which
is absent, and holds no fixture for this op.
GPU: the HIP assembly + device fp64 Cholesky against the oracle.  Both sides
solve in fp64 and round the step to fp32: relative 2-norm error <= 1e-5."""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import oracle


def make_pgo(n, r, seed, chain=True):
    """Pose graph over n Sim3 poses: odometry chain (i, i+1) plus random loop
    edges, 7x7 Jacobian blocks near +-identity like optim_utils.py's
    J_Ginv_i / J_Ginv_j, residuals N(0, 0.1)."""
    rng = np.random.default_rng(seed)
    ii, jj = [], []
    if chain:
        for i in range(n - 1):
            ii.append(i)
            jj.append(i + 1)
    while len(ii) < r:
        a, b = rng.integers(0, n, 2)
        if a != b:
            ii.append(a)
            jj.append(b)
    ii = np.array(ii, np.int64)
    jj = np.array(jj, np.int64)
    m = len(ii)
    eye = np.eye(7, dtype=np.float32)
    Ji = (-eye + 0.1 * rng.standard_normal((m, 7, 7))).astype(np.float32)
    Jj = (eye + 0.1 * rng.standard_normal((m, 7, 7))).astype(np.float32)
    res = (0.1 * rng.standard_normal((m, 7))).astype(np.float32)
    return Ji, Jj, ii, jj, res


def sparse_reference(Ji, Jj, ii, jj, res, ep, lm, freen):
    r = len(ii)
    n = int(max(ii.max(), jj.max())) + 1
    rows, cols, vals = [], [], []
    for x in range(r):  # ba.cpp:146-157
        for k in range(7):
            for l in range(7):
                rows += [x * 7 + k, x * 7 + k]
                cols += [ii[x] * 7 + l, jj[x] * 7 + l]
                vals += [float(Ji[x, k, l]), float(Jj[x, k, l])]
    J = sp.csr_matrix((vals, (rows, cols)), shape=(7 * r, 7 * n))
    v = res.reshape(-1).astype(np.float64)
    b = -(J.T @ v)
    A = (J.T @ J).tocsc()
    A.setdiag(A.diagonal() + A.diagonal() * float(np.float32(lm)) + float(np.float32(ep)))
    f = freen * 7
    delta = np.zeros(7 * n)
    if f < 0:
        f = 7 * n
    if f > 0:
        delta[:f] = spla.spsolve(A[:f, :f].tocsc(), b[:f])
    return delta.astype(np.float32).reshape(n, 7)


@pytest.mark.parametrize("n,r,freen", [(6, 8, 5), (12, 30, -1), (20, 40, 12), (5, 4, 0)])
def test_oracle_matches_sparse_restatement(n, r, freen):
    Ji, Jj, ii, jj, res = make_pgo(n, r, seed=n + r)
    a = oracle.solve_system(Ji, Jj, ii, jj, res, 1e-4, 1e-4, freen)
    b = sparse_reference(Ji, Jj, ii, jj, res, 1e-4, 1e-4, freen)
    assert a.shape == (n, 7)
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    if 0 <= freen < n:
        assert np.all(a[freen:] == 0)


def test_oracle_rejects_self_edge():
    Ji, Jj, ii, jj, res = make_pgo(4, 4, seed=1)
    jj[2] = ii[2]
    with pytest.raises(ValueError):
        oracle.solve_system(Ji, Jj, ii, jj, res, 1e-4, 1e-4, -1)


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.mark.gpu
@pytest.mark.parametrize("n,r,freen", [(6, 8, 5), (12, 30, -1), (20, 40, 12), (5, 4, 0),
                                       (300, 900, 299), (400, 1000, -1)])
def test_solve_system_gpu(gpu, n, r, freen):
    import torch
    import dpvo_amd

    cb = dpvo_amd.load_extension("cuda_ba")
    Ji, Jj, ii, jj, res = make_pgo(n, r, seed=n + r)
    ep, lm = 1e-4, 1e-4
    want = oracle.solve_system(Ji, Jj, ii, jj, res, ep, lm, freen)
    t = lambda a: torch.from_numpy(a).to(gpu)
    out = cb.solve_system(t(Ji), t(Jj), t(ii), t(jj), t(res), ep, lm, freen)
    assert isinstance(out, list) and len(out) == 1
    got = out[0]
    assert got.dtype == torch.float32 and tuple(got.shape) == (n, 7) and got.device == gpu
    got = got.cpu().numpy()
    assert _rel(got, want) <= 1e-5, _rel(got, want)
    if 0 <= freen < n:
        assert np.all(got[freen:] == 0)


@pytest.mark.gpu
def test_solve_system_gpu_errors(gpu):
    import torch
    import dpvo_amd

    cb = dpvo_amd.load_extension("cuda_ba")
    Ji, Jj, ii, jj, res = make_pgo(4, 4, seed=3)
    jj[1] = ii[1]
    t = lambda a: torch.from_numpy(a).to(gpu)
    with pytest.raises(RuntimeError, match="ii == jj"):
        cb.solve_system(t(Ji), t(Jj), t(ii), t(jj), t(res), 1e-4, 1e-4, -1)
    with pytest.raises(RuntimeError):
        cb.solve_system(t(Ji), t(Jj), t(ii), t(jj[:2]), t(res), 1e-4, 1e-4, -1)
