"""GPU parity against the reference's OWN outputs (tests/golden/, written by
oracle/make_golden.py running /root/reference's Python in the build
container), on the exact product paths the bench runs:

* P-TRANSFORM: dpvo_amd.projective_ops.transform(..., jacobian=True) on the
  HIP lietorch vs dpvo/projective_ops.py:53-113 (coords, valid, Ji, Jj, Jz).
* F-BA: cuda_ba.forward (1 iteration) vs dpvo/ba.py BA (88-297) run in fp64
  on inputs where its divergences from ba_cuda.cu are inert (ep=1.0, CUDA
  bounds; SURVEY 8(a) A-BA-PY) -- the reference-run vectors directly, not
  through the oracle.
* A-CORR channels-last (corr_nhwc.hip, the matrix-core path) vs the 128-channel
  reference loop fixture corr_loop_a (correlation_kernel.py:388-458).
* A-CORR channels-last at FULL cfg2 size (2048 edges, 120x160, levels
  [1,2,4,8]) vs the oracle per level.

Tolerances are written per test (fp32 work; north_star: 1e-4 rel)."""
import numpy as np
import pytest
import torch
from conftest import golden

import oracle

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("name", ["ba_py_a", "ba_py_b"])
def test_transform_matches_reference_jacobians(gpu, name):
    from dpvo_amd import projective_ops as pops
    from dpvo_amd.lietorch import SE3

    z = golden(name)
    poses = SE3(_t(z["poses"], gpu)[None])
    patches = _t(z["patches"], gpu)[None]
    intr = _t(z["intrinsics"], gpu)[None]
    ii, jj, kk = (_t(z[k], gpu) for k in ("ii", "jj", "kk"))
    coords, valid, (Ji, Jj, Jz) = pops.transform(poses, patches, intr, ii, jj, kk, jacobian=True)
    # fp32 geometry; the reference ran the same fp32 op sequence on the CPU
    np.testing.assert_allclose(coords[0].cpu().numpy(), z["tr_coords"], rtol=0, atol=1e-4)
    np.testing.assert_array_equal(valid[0].cpu().numpy(), z["tr_valid"])
    for got, ref in ((Ji, "tr_Ji"), (Jj, "tr_Jj"), (Jz, "tr_Jz")):
        r = z[ref]
        np.testing.assert_allclose(got[0].cpu().numpy(), r, rtol=1e-4,
                                   atol=1e-5 * max(1.0, np.abs(r).max()), err_msg=ref)


@pytest.mark.parametrize("name", ["ba_py_a", "ba_py_b"])
def test_ba_matches_reference_ba_py(gpu, name):
    import dpvo_amd

    cb = dpvo_amd.load_extension("cuda_ba")
    z = golden(name)
    t0, t1 = int(z["t0"]), int(z["t1"])
    poses, patches = _t(z["poses"], gpu).clone(), _t(z["patches"], gpu).clone()
    M = z["patches"].shape[0] // z["poses"].shape[0]
    cb.forward(poses, patches, _t(z["intrinsics"], gpu), _t(z["target"], gpu), _t(z["weight"], gpu),
               torch.tensor([float(z["lmbda"])], device=gpu), _t(z["ii"], gpu), _t(z["jj"], gpu),
               _t(z["kk"], gpu), M, t0, t1, 1, False)
    # a non-zero BA status (e.g. a spin-wait timeout, bit 16) raises here with
    # its cause, instead of surfacing only as a numeric mismatch below
    cb.check_status(poses)
    P, K = poses.cpu().numpy(), patches.cpu().numpy()
    # tight against the reference's fp64 run (our reductions/solve are fp64)
    np.testing.assert_allclose(P, z["out_poses64"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(K, z["out_patches64"], rtol=1e-4, atol=2e-5)
    # pose deltas within 1e-4 relative (north_star)
    d = P.astype(np.float64) - z["poses"]
    dr = z["out_poses64"] - z["poses"]
    assert np.linalg.norm(d - dr) <= 1e-4 * np.linalg.norm(dr) + 1e-6
    # loose against its fp32 run (the reference's own fp32 noise)
    np.testing.assert_allclose(P, z["out_poses"], rtol=0, atol=5e-5)


def test_channels_last_corr_matches_reference_loop(gpu):
    from dpvo_amd import altcorr, synthetic

    z = golden("corr_loop_a")  # C = 128: the MFMA path's shape
    R = int(z["radius"])
    f2 = _t(z["fmap2"], gpu)
    out = altcorr.corr_levels(_t(z["fmap1"], gpu), [synthetic.channels_last(f2)], _t(z["coords"], gpu),
                              _t(z["ii"], gpu), _t(z["jj"], gpu), R, scales=(1,))
    M = z["coords"].shape[1]
    got = out.view(1, M, 2 * R + 1, 2 * R + 1, 3, 3).cpu().numpy()
    ref = z["out"]
    assert np.abs(got - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())


def test_channels_last_cfg2_full_size_matches_oracle(gpu):
    """The bench's exact A-CORR launch shape: 2048 edges, 128 channels,
    120x160 level 1, levels [1,2,4,8], channels-last ring of 36 frames,
    coords from the product reprojection, XCD edge order on."""
    from dpvo_amd import altcorr, fastba, synthetic

    G = synthetic.make_config("cfg2", seed=0)
    D = G.to(gpu)
    mem, levels = 36, (1, 2, 4, 8)
    pyr = synthetic.make_features(mem=mem, C=128, levels=levels, seed=0, device=gpu)
    pyr_cl = [synthetic.channels_last(p) for p in pyr]
    gmap = 0.25 * torch.randn(1, mem * G.M, 128, 3, 3, device=gpu,
                              generator=torch.Generator(device=gpu).manual_seed(3))
    coords, order = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem)
    kk1, jj1 = D.kk % (mem * G.M), D.jj % mem
    out = altcorr.corr_levels(gmap, pyr_cl, coords, kk1, jj1, 3, levels, order=order)
    out = out.view(1, G.E, 7, 7, 3, 3, len(levels)).cpu().numpy()
    g, co = gmap.cpu().numpy(), coords.cpu().numpy()
    k, j = kk1.cpu().numpy(), jj1.cpu().numpy()
    for l, s in enumerate(levels):
        ref = oracle.corr_fwd(g, pyr[l].cpu().numpy(), co / s, k, j, 3)
        err = np.abs(out[..., l] - ref).max()
        assert err <= 1e-5 * max(1.0, np.abs(ref).max()), (s, err)
