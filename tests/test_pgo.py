"""cuda_ba.solve_system (Sim3 pose-graph solve, dpvo/fastba/ba.cpp:120-180).

CPU: the numpy oracle against an independent scipy.sparse formulation that
follows ba.cpp literally (triplets -> J, Jt*J, diagonal damping, solve of the
top-left block).  Parity unpinned otherwise: the reference needs Eigen, which
is absent, and holds no fixture for this op.
GPU: the structured HIP solve (deterministic block assembly, block-tridiagonal
segment sweeps, dense border) against the oracle.  Both sides solve in fp64
and round the step to fp32: relative 2-norm error <= 1e-5 (1e-4 on the
ep = 0 / lm = 1e-6 gauge-deficient systems the loop-closure caller builds,
optim_utils.py:211-229, whose condition number is ~1e7)."""
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


def make_loop_graph(n, loops, seed, gauge=False):
    """Loop-closure shaped graph (long_term.py / optim_utils.py:164-189): the
    odometry chain plus `loops` long edges between a recent and an old pose.
    gauge=True: J_Ginv_j = -J_Ginv_i exactly, so J^T J has the global null
    space of a relative-pose residual (the caller passes freen = -1)."""
    rng = np.random.default_rng(seed)
    ii = list(range(n - 1))
    jj = list(range(1, n))
    for _ in range(loops):
        a = int(rng.integers(n // 2, n))
        b = int(rng.integers(0, max(a - 2, 1)))
        if a - b > 1:
            ii.append(a)
            jj.append(b)
    ii = np.array(ii, np.int64)
    jj = np.array(jj, np.int64)
    m = len(ii)
    eye = np.eye(7, dtype=np.float32)
    Ji = (-eye + 0.1 * rng.standard_normal((m, 7, 7))).astype(np.float32)
    Jj = -Ji if gauge else (eye + 0.1 * rng.standard_normal((m, 7, 7))).astype(np.float32)
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


def _plan(ii, jj, nf):
    import ctypes
    import dpvo_amd

    lib = dpvo_amd.c_abi()
    ii = np.ascontiguousarray(ii, np.int64)
    jj = np.ascontiguousarray(jj, np.int64)
    P = ctypes.POINTER(ctypes.c_int64)
    n = ctypes.c_int64(0)
    assert lib.dpvo_pgo_plan(ii.ctypes.data_as(P), jj.ctypes.data_as(P), len(ii), nf, None, 0,
                             ctypes.byref(n)) == 0
    plan = np.zeros(n.value, np.int64)
    assert lib.dpvo_pgo_plan(ii.ctypes.data_as(P), jj.ctypes.data_as(P), len(ii), nf,
                             plan.ctypes.data_as(P), n.value, ctypes.byref(n)) == 0
    return plan


def test_pgo_plan_structure():
    """Host plan of the structured solve: border = endpoints of long edges
    inside the free range, segments = the runs of the other poses with their
    neighbouring border poses, one task per distinct 7x7 block with its edges
    in ascending order."""
    # chain 0..9, long edges 8-2 and 9-7, a duplicate chain edge 4-5, an edge to
    # fixed pose 11 (free range nf = 10)
    ii = np.array([0, 1, 2, 3, 4, 5, 6, 7, 8, 8, 9, 5, 9], np.int64)
    jj = np.array([1, 2, 3, 4, 5, 6, 7, 8, 9, 2, 7, 4, 11], np.int64)
    plan = _plan(ii, jj, 10)
    nf, ntask, nseg, m = plan[:4]
    assert nf == 10 and m == 4  # border poses 2, 7, 8, 9
    segs = plan[plan[6]:plan[6] + 4 * nseg].reshape(nseg, 4)
    assert segs.tolist() == [[0, 1, -1, 0], [3, 6, 0, 1]]
    bord = plan[plan[7]:plan[7] + 3 * m].reshape(m, 3)
    assert bord.tolist() == [[2, 0, 1], [7, 1, -1], [8, -1, -1], [9, -1, -1]]
    tasks = plan[plan[4]:plan[4] + 8 * ntask].reshape(ntask, 8)
    contrib = plan[plan[5]:plan[6]]
    # 10 diagonal tasks, then one per distinct pair inside the free range
    assert ntask == 10 + 11  # 9 chain pairs + 8-2 + 9-7 (the duplicate 4-5 merges)
    diag9 = tasks[9]
    assert list(contrib[diag9[2]:diag9[3]]) == [8, 10, 12]  # edges touching pose 9, ascending
    pair54 = [t for t in tasks[10:] if (t[0], t[1]) == (5, 4)]
    assert len(pair54) == 1 and list(contrib[pair54[0][2]:pair54[0][3]]) == [4, 11]
    # an invalid graph is rejected on the host
    import ctypes
    import dpvo_amd

    P = ctypes.POINTER(ctypes.c_int64)
    bad = np.array([3], np.int64)
    n = ctypes.c_int64(0)
    assert dpvo_amd.c_abi().dpvo_pgo_plan(bad.ctypes.data_as(P), bad.ctypes.data_as(P), 1, 4,
                                          None, 0, ctypes.byref(n)) == 1


def _gpu_solve(gpu, Ji, Jj, ii, jj, res, ep, lm, freen):
    import torch
    import dpvo_amd

    cb = dpvo_amd.load_extension("cuda_ba")
    t = lambda a: torch.from_numpy(a).to(gpu)
    return cb.solve_system(t(Ji), t(Jj), t(ii), t(jj), t(res), ep, lm, freen)[0].cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("n,loops,freen", [(2, 0, -1), (3, 1, -1), (40, 0, -1), (40, 3, -1),
                                           (60, 5, 45), (200, 12, -1), (500, 20, 480),
                                           (2000, 30, -1)])
def test_solve_system_loop_graphs_gpu(gpu, n, loops, freen):
    Ji, Jj, ii, jj, res = make_loop_graph(n, loops, seed=n + loops)
    want = sparse_reference(Ji, Jj, ii, jj, res, 1e-4, 1e-4, freen)
    got = _gpu_solve(gpu, Ji, Jj, ii, jj, res, 1e-4, 1e-4, freen)
    assert got.shape == want.shape
    assert _rel(got, want) <= 1e-5, _rel(got, want)
    if 0 <= freen < n:
        assert np.all(got[freen:] == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("n,loops", [(30, 2), (300, 8)])
def test_solve_system_gauge_deficient_gpu(gpu, n, loops):
    """The caller's conditioning: ep = 0, lm = 1e-6, freen = -1 and a
    relative-pose Jacobian (7-dim null space of J^T J): only the lm-scaled
    diagonal makes the system definite (optim_utils.py:211)."""
    Ji, Jj, ii, jj, res = make_loop_graph(n, loops, seed=7 * n, gauge=True)
    want = sparse_reference(Ji, Jj, ii, jj, res, 0.0, 1e-6, -1)
    got = _gpu_solve(gpu, Ji, Jj, ii, jj, res, 0.0, 1e-6, -1)
    assert np.all(np.isfinite(got))
    assert _rel(got, want) <= 1e-4, _rel(got, want)


@pytest.mark.gpu
def test_solve_system_deterministic_and_host_inputs(gpu):
    """Fixed-order assembly: repeated calls are bit-identical.  Host (CPU)
    tensors are accepted as the reference's caller passes them (long_term.py
    moves the poses to the CPU) and the step comes back on the CPU."""
    import torch
    import dpvo_amd

    cb = dpvo_amd.load_extension("cuda_ba")
    Ji, Jj, ii, jj, res = make_loop_graph(300, 10, seed=5)
    a = _gpu_solve(gpu, Ji, Jj, ii, jj, res, 1e-4, 1e-4, -1)
    b = _gpu_solve(gpu, Ji, Jj, ii, jj, res, 1e-4, 1e-4, -1)
    assert np.array_equal(a, b)
    t = torch.from_numpy
    c = cb.solve_system(t(Ji), t(Jj), t(ii), t(jj), t(res), 1e-4, 1e-4, -1)[0]
    assert c.device.type == "cpu" and np.array_equal(c.numpy(), a)


@pytest.mark.gpu
def test_solve_system_unconstrained_pose_raises(gpu):
    """A free pose without edges and ep = 0 leaves a zero pivot: RuntimeError
    (Eigen's result is undefined there; the dense path raised the same)."""
    Ji, Jj, ii, jj, res = make_loop_graph(10, 0, seed=1)
    keep = ~((ii == 4) | (jj == 4))  # pose 4 loses both chain edges
    args = (Ji[keep], Jj[keep], ii[keep], jj[keep], res[keep])
    with pytest.raises(RuntimeError, match="not positive definite"):
        _gpu_solve(gpu, *args, 0.0, 1e-6, -1)
