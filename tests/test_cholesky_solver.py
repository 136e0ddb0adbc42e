"""CholeskySolver (dpvo/ba.py:13-38) on this build's batched HIP SPD solve
(spd_solve.hip): forward vs a direct fp64 solve (LDS-resident and HBM-resident
sizes, fp32 and fp64), the factor vs torch.linalg.cholesky, info = the first
failed column as cholesky_ex reports it, backward vs torch.autograd.gradcheck
(fp64), the failure path (zeros forward, no gradient), block_solve against a
dense restatement of dpvo/ba.py:67-77, and the CPU-tensor refusal."""
import pytest
import torch

from dpvo_amd.ba import CholeskySolver, block_solve


def _spd(n, k, dev, dtype=torch.float64, seed=0):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(2, n, n, generator=g, dtype=dtype)
    H = A @ A.transpose(-1, -2) + n * torch.eye(n, dtype=dtype)
    b = torch.randn(2, n, k, generator=g, dtype=dtype)
    return H.to(dev), b.to(dev)


@pytest.mark.gpu
def test_forward_matches_direct_solve(gpu):
    H, b = _spd(30, 2, gpu)
    x = CholeskySolver.apply(H, b)
    torch.testing.assert_close(x, torch.linalg.solve(H, b), rtol=1e-10, atol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,dtype,tol", [(6, 1, torch.float64, 1e-10), (66, 3, torch.float64, 1e-10),
                                           (150, 2, torch.float64, 1e-9),  # HBM working copy
                                           (66, 1, torch.float32, 2e-4), (200, 1, torch.float32, 5e-4),
                                           (210, 1, torch.float32, 5e-4),  # fp32 HBM working copy
                                           (120, 300, torch.float32, 5e-4)])  # k pushes it out of LDS
def test_spd_solve_matches_dense(gpu, n, k, dtype, tol):
    from dpvo_amd.ba import _cuda_ba

    H, b = _spd(n, k, gpu, dtype=dtype, seed=n)
    # the kernel reads the lower triangle only (cholesky_ex upper=False)
    Hu = H + torch.triu(torch.full_like(H, 7.0), diagonal=1)
    x, L, info = _cuda_ba.spd_solve(Hu, b)
    assert info.shape == (2,) and int(info.abs().sum()) == 0
    ref = torch.linalg.solve(H.double(), b.double())
    err = ((x.double() - ref).norm() / ref.norm()).item()
    assert err < tol, err
    Lref = torch.linalg.cholesky(H.double())
    assert ((L.double() - Lref).norm() / Lref.norm()).item() < tol
    assert torch.count_nonzero(torch.triu(L, diagonal=1)) == 0
    # solve with the stored factor (the backward's cholesky_solve)
    x2 = _cuda_ba.spd_solve_factored(L, b)
    assert ((x2.double() - ref).norm() / ref.norm()).item() < tol


@pytest.mark.gpu
def test_spd_info_is_first_failed_column(gpu):
    from dpvo_amd.ba import _cuda_ba

    H, b = _spd(10, 1, gpu)
    H[1, 4, :] = 0
    H[1, :, 4] = 0  # column 4 of item 1 has no pivot
    x, L, info = _cuda_ba.spd_solve(H, b)
    _, ref_info = torch.linalg.cholesky_ex(H.cpu())
    assert info.cpu().tolist() == ref_info.tolist() == [0, 5]
    assert torch.count_nonzero(x[1]) == 0 and torch.count_nonzero(x[0]) > 0


@pytest.mark.gpu
def test_block_solve_matches_dense_reference(gpu):
    from dpvo_amd.ba import block_matmul

    g = torch.Generator().manual_seed(3)
    J = torch.randn(2, 4, 4, 6, 6, generator=g, dtype=torch.float64)
    A = block_matmul(J.to(gpu), J.permute(0, 2, 1, 4, 3).contiguous().to(gpu))  # SPD blocks
    B = torch.randn(2, 4, 1, 6, 1, generator=g, dtype=torch.float64).to(gpu)
    X = block_solve(A, B)
    # dpvo/ba.py:67-77 restated densely
    Ad = A.permute(0, 1, 3, 2, 4).reshape(2, 24, 24)
    Bd = B.permute(0, 1, 3, 2, 4).reshape(2, 24, 1)
    Ad = Ad + (1.0 + 1e-4 * Ad) * torch.eye(24, device=gpu, dtype=torch.float64)
    ref = torch.linalg.solve(Ad, Bd).reshape(2, 4, 6, 1, 1).permute(0, 1, 3, 2, 4)
    torch.testing.assert_close(X, ref, rtol=1e-9, atol=1e-9)
    # block_matmul vs the dense product
    Jd = J.permute(0, 1, 3, 2, 4).reshape(2, 24, 24)
    torch.testing.assert_close(A.cpu().permute(0, 1, 3, 2, 4).reshape(2, 24, 24), Jd @ Jd.transpose(1, 2))


@pytest.mark.gpu
def test_backward_gradcheck(gpu):
    H, b = _spd(8, 1, gpu)
    H.requires_grad_()
    b.requires_grad_()
    # the reference's backward treats H as a free (not symmetric-constrained)
    # matrix: dH = -x dz^T; gradcheck on the symmetric part fed through
    assert torch.autograd.gradcheck(lambda h, v: CholeskySolver.apply(0.5 * (h + h.transpose(-1, -2)), v),
                                    (H, b), eps=1e-6, atol=1e-5)


@pytest.mark.gpu
def test_failure_returns_zeros_and_no_grad(gpu):
    H, b = _spd(6, 1, gpu)
    H = -H  # not positive definite
    H.requires_grad_()
    x = CholeskySolver.apply(H, b)
    assert torch.count_nonzero(x) == 0
    x.sum().backward()
    assert H.grad is None


@pytest.mark.gpu
def test_block_solve_shapes(gpu):
    A = torch.randn(1, 3, 3, 6, 6, device=gpu, dtype=torch.float64)
    A = A + A.permute(0, 2, 1, 4, 3)
    A = A + 50 * torch.eye(6, device=gpu, dtype=torch.float64).view(1, 1, 1, 6, 6) * \
        torch.eye(3, device=gpu, dtype=torch.float64).view(1, 3, 3, 1, 1)
    B = torch.randn(1, 3, 1, 6, 1, device=gpu, dtype=torch.float64)
    X = block_solve(A, B)
    assert X.shape == (1, 3, 1, 6, 1)


def test_cpu_tensors_are_refused():
    H, b = _spd(4, 1, "cpu")
    with pytest.raises(RuntimeError, match="GPU"):
        CholeskySolver.apply(H, b)
