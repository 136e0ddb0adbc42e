"""GPU parity of altcorr (A-CORR, A-CORR-BWD, A-PATCH, A-PATCH-BWD) through the
cuda_corr extension (-> C ABI -> HIP kernels) against the reference's golden
vectors and the oracle.

Tolerances (fp32): the reference accumulates the 128-long dot in fp32 in an
arbitrary order, the oracle in fp64; elementwise |gpu - ref| <= 1e-5 *
max(1, |ref|_max) covers fp32 summation noise (north_star: "fp32 correlation
volumes within 1e-4 rel")."""
import numpy as np
import pytest
import torch
from conftest import golden

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cc(gpu):
    import dpvo_amd

    return dpvo_amd.load_extension("cuda_corr")


def _t(a, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t.to(dtype) if dtype is not None else t


def _close(out, ref, tol=1e-5):
    ref = np.asarray(ref, np.float64)
    out = np.asarray(out, np.float64)
    assert out.shape == ref.shape
    err = np.abs(out - ref).max() if ref.size else 0.0
    assert err <= tol * max(1.0, np.abs(ref).max() if ref.size else 1.0), err


@pytest.mark.parametrize("name", ["corr_loop_a", "corr_loop_b", "corr_loop_c", "corr_gs_a"])
def test_forward_matches_reference_golden(cc, gpu, name):
    z = golden(name)
    out, = cc.forward(_t(z["fmap1"], gpu), _t(z["fmap2"], gpu), _t(z["coords"], gpu),
                      _t(z["ii"], gpu), _t(z["jj"], gpu), int(z["radius"]))
    _close(out.cpu().numpy(), z["out"], 1e-5 if name != "corr_gs_a" else 2e-5)


def _case(seed, B=1, M=37, C=128, N1=9, N2=4, H2=24, W2=32, p=3, R=3, spread=0.3, far=0.1,
          Hp=None, Wp=None):
    r = np.random.default_rng(seed)
    Hp = Hp or p
    Wp = Wp or p
    f1 = (0.25 * r.standard_normal((B, N1, C, Hp, Wp))).astype(np.float32)
    f2 = (0.25 * r.standard_normal((B, N2, C, H2, W2))).astype(np.float32)
    cx = r.uniform(-4, W2 + 4, (B, M, 1, 1))
    cy = r.uniform(-4, H2 + 4, (B, M, 1, 1))
    gx = np.arange(Wp)[None, None, None, :] - Wp // 2 + spread * r.standard_normal((B, M, Hp, Wp))
    gy = np.arange(Hp)[None, None, :, None] - Hp // 2 + spread * r.standard_normal((B, M, Hp, Wp))
    co = np.stack([cx + gx, cy + gy], 2).astype(np.float32)
    co[:, : int(far * M), 0] += 5 * W2  # windows completely outside the map
    ii = r.integers(0, N1, M)
    jj = r.integers(0, N2, M)
    return f1, f2, co, ii, jj, R


@pytest.mark.parametrize("kw", [
    dict(),                                  # DPVO shape: p=3, R=3, C=128
    dict(R=0), dict(R=1), dict(R=2), dict(R=7),
    dict(p=1), dict(p=2), dict(p=4),         # other exact patch sizes
    dict(Hp=2, Wp=3),                        # non-square patch -> generic path
    dict(spread=4.0),                        # windows too spread for the box
    dict(B=2, M=11),                         # batch
    dict(C=37, M=5),                         # channel tail (C % 4 != 0)
    dict(H2=5, W2=6, M=21),                  # tiny map: every window clipped
])
def test_forward_matches_oracle(cc, gpu, kw):
    f1, f2, co, ii, jj, R = _case(1, **kw)
    out, = cc.forward(_t(f1, gpu), _t(f2, gpu), _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R)
    _close(out.cpu().numpy(), oracle.corr_fwd(f1, f2, co, ii, jj, R))


def test_forward_cfg2_full_size(cc, gpu):
    # full BASELINE cfg2 edge count against the oracle (both levels of DPVO.corr)
    from dpvo_amd import synthetic

    G = synthetic.make_config("cfg2", seed=0)
    pyr = synthetic.make_features(mem=12, levels=(1, 4), seed=0, device=gpu)
    r = np.random.default_rng(0)
    gmap = (0.25 * r.standard_normal((1, 12 * 96, 128, 3, 3))).astype(np.float32)
    coords = oracle.reproject(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(),
                              G.ii.numpy(), G.jj.numpy(), G.kk.numpy())
    for lvl, s in enumerate((1, 4)):
        co = (coords / s).astype(np.float32)
        f2 = pyr[lvl].cpu().numpy()
        out, = cc.forward(_t(gmap, gpu), pyr[lvl], _t(co, gpu), _t(G.kk.numpy(), gpu),
                          _t(G.jj.numpy(), gpu), 3)
        _close(out.cpu().numpy(), oracle.corr_fwd(gmap, f2, co, G.kk.numpy(), G.jj.numpy(), 3))


def test_forward_is_deterministic(cc, gpu):
    f1, f2, co, ii, jj, R = _case(2, M=200)
    args = (_t(f1, gpu), _t(f2, gpu), _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R)
    a, = cc.forward(*args)
    b, = cc.forward(*args)
    assert torch.equal(a, b)


def test_forward_levels_equals_per_level_calls(cc, gpu):
    from dpvo_amd import altcorr

    f1, f2, co, ii, jj, R = _case(3, M=64, H2=40, W2=48)
    f1, co, ii, jj = _t(f1, gpu), _t(co, gpu), _t(ii, gpu), _t(jj, gpu)
    lv1 = _t(f2, gpu)
    lv2 = torch.nn.functional.avg_pool2d(lv1[0], 4, 4).unsqueeze(0).contiguous()
    fused = altcorr.corr_levels(f1, [lv1, lv2], co, ii, jj, R, scales=(1, 4))
    c1, = cc.forward(f1, lv1, co / 1, ii, jj, R)
    c2, = cc.forward(f1, lv2, co / 4, ii, jj, R)
    ref = torch.stack([c1, c2], -1).view(1, len(ii), -1)  # dpvo.py:465
    # same per-level arithmetic; allow only last-bit differences from code
    # generation of the two launch shapes
    err = (fused - ref).abs().max().item()
    assert err <= 1e-6 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("dtype", [torch.float16, torch.float64])
def test_forward_other_dtypes(cc, gpu, dtype):
    f1, f2, co, ii, jj, R = _case(4, M=23)
    f1h, f2h = torch.from_numpy(f1).to(dtype), torch.from_numpy(f2).to(dtype)
    out, = cc.forward(f1h.to(gpu), f2h.to(gpu), _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R)
    assert out.dtype == dtype
    ref = oracle.corr_fwd(f1h.double().numpy(), f2h.double().numpy(), co, ii, jj, R)
    _close(out.double().cpu().numpy(), ref, 2e-3 if dtype == torch.float16 else 1e-6)


def test_forward_empty(cc, gpu):
    f1, f2, co, ii, jj, R = _case(5, M=3)
    out, = cc.forward(_t(f1, gpu), _t(f2, gpu), _t(co[:, :0], gpu), _t(ii[:0], gpu),
                      _t(jj[:0], gpu), R)
    assert out.shape == (1, 0, 7, 7, 3, 3)


@pytest.mark.parametrize("kw", [dict(), dict(spread=4.0), dict(R=1, M=9)])
def test_backward_matches_oracle(cc, gpu, kw):
    f1, f2, co, ii, jj, R = _case(6, **{**dict(M=19, C=32), **kw})
    Dp = 2 * R + 1
    G = np.random.default_rng(7).standard_normal((1, len(ii), Dp, Dp, 3, 3)).astype(np.float32)
    g1, g2 = cc.backward(_t(f1, gpu), _t(f2, gpu), _t(co, gpu), _t(ii, gpu), _t(jj, gpu),
                         _t(G, gpu), R)
    r1, r2 = oracle.corr_bwd(f1, f2, co, ii, jj, G, R)
    _close(g1.cpu().numpy(), r1, 1e-5)
    _close(g2.cpu().numpy(), r2, 1e-5)


@pytest.mark.parametrize("name", ["patchify_a", "patchify_b", "patchify_c"])
def test_patchify_matches_reference_golden(cc, gpu, name):
    z = golden(name)
    R = int(z["radius"])
    net, co = _t(z["net"], gpu), _t(z["coords"], gpu)
    zero, = cc.patchify_forward(net, co, R)
    clamp, = cc.patchify_forward_clamped(net, co, R)
    np.testing.assert_array_equal(zero.cpu().numpy(), z["out_zero"])
    np.testing.assert_array_equal(clamp.cpu().numpy(), z["out_clamp"])


@pytest.mark.parametrize("clamp", [False, True])
def test_patchify_backward_matches_oracle(cc, gpu, clamp):
    r = np.random.default_rng(8)
    net = r.standard_normal((1, 16, 20, 24)).astype(np.float32)
    co = np.stack([r.uniform(-3, 27, (1, 40)), r.uniform(-3, 23, (1, 40))], -1).astype(np.float32)
    G = r.standard_normal((1, 40, 16, 4, 4)).astype(np.float32)
    fn = cc.patchify_backward_clamped if clamp else cc.patchify_backward
    g, = fn(_t(net, gpu), _t(co, gpu), _t(G, gpu), 1)
    _close(g.cpu().numpy(), oracle.patchify_bwd(net.shape, co, G, 1, clamp), 1e-5)


def test_autograd_wrappers(gpu):
    # dpvo_amd.altcorr mirrors dpvo/altcorr/correlation.py (CorrLayer / PatchLayer)
    from dpvo_amd import altcorr

    f1, f2, co, ii, jj, R = _case(9, M=12, C=16)
    a = _t(f1, gpu).requires_grad_()
    b = _t(f2, gpu).requires_grad_()
    out = altcorr.corr(a, b, _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R)
    G = torch.randn_like(out)
    (out * G).sum().backward()
    r1, r2 = oracle.corr_bwd(f1, f2, co, ii, jj, G.cpu().numpy(), R)
    _close(a.grad.cpu().numpy(), r1)
    _close(b.grad.cpu().numpy(), r2)
    net = torch.randn(1, 8, 20, 20, device=gpu)
    c2 = torch.rand(1, 10, 2, device=gpu) * 18 + 1
    p = altcorr.patchify(net, c2, 1)
    assert p.shape == (1, 10, 8, 3, 3)


# ---- channels-last pyramid: matrix-core path (corr_nhwc.hip) ----
@pytest.mark.parametrize("kw", [dict(), dict(spread=4.0), dict(far=0.3),
                                dict(M=130, H2=12, W2=14)])
@pytest.mark.parametrize("levels", [(1,), (1, 4), (1, 2, 4, 8)])
def test_channels_last_levels_match_oracle(gpu, kw, levels):
    from dpvo_amd import altcorr, synthetic

    f1, f2, co, ii, jj, R = _case(11, **{**dict(M=67, C=128, H2=40, W2=48), **kw})
    lv1 = _t(f2, gpu)
    pyr = [lv1 if s == 1 else torch.nn.functional.avg_pool2d(lv1[0], s, s).unsqueeze(0)
           for s in levels]
    pyr_cl = [synthetic.channels_last(p) for p in pyr]
    out = altcorr.corr_levels(_t(f1, gpu), pyr_cl, _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R,
                              scales=levels)
    out = out.view(1, len(ii), 2 * R + 1, 2 * R + 1, 3, 3, len(levels)).cpu().numpy()
    for l, s in enumerate(levels):
        ref = oracle.corr_fwd(f1, pyr[l].cpu().numpy(), co / s, ii, jj, R)
        _close(out[..., l], ref, 1e-5)


def test_channels_last_equals_nchw_path(cc, gpu):
    from dpvo_amd import altcorr, synthetic

    f1, f2, co, ii, jj, R = _case(12, M=200, C=128, H2=60, W2=80)
    lv1 = _t(f2, gpu)
    pyr = [lv1, torch.nn.functional.avg_pool2d(lv1[0], 4, 4).unsqueeze(0).contiguous()]
    a = altcorr.corr_levels(_t(f1, gpu), pyr, _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R, (1, 4))
    b = altcorr.corr_levels(_t(f1, gpu), [synthetic.channels_last(p) for p in pyr], _t(co, gpu),
                            _t(ii, gpu), _t(jj, gpu), R, (1, 4))
    err = (a - b).abs().max().item()
    assert err <= 1e-5 * max(1.0, a.abs().max().item()), err


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_forward_channels_last_level_matches_oracle(cc, gpu, dtype):
    """cuda_corr.forward (the reference's per-level entry, dpvo.py:462-465)
    on a channels-last level -- a DPVO pyramid allocated channels-last
     -- takes the matrix-core kernel and returns the
    reference's [B, M, 7, 7, p, p] in the fmap dtype."""
    from dpvo_amd import synthetic

    f1, f2, co, ii, jj, R = _case(13, M=150, C=128, H2=40, W2=48)
    if dtype == torch.float16:  # compare on the fp16-rounded inputs
        f1 = f1.astype(np.float16).astype(np.float32)
        f2 = f2.astype(np.float16).astype(np.float32)
    lv = synthetic.channels_last(_t(f2, gpu, dtype))
    assert not lv.is_contiguous()
    out, = cc.forward(_t(f1, gpu, dtype), lv, _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R)
    assert out.dtype == dtype and out.shape == (1, len(ii), 2 * R + 1, 2 * R + 1, 3, 3)
    ref = oracle.corr_fwd(f1, f2, co, ii, jj, R)
    _close(out.float().cpu().numpy(), ref, 1e-5 if dtype == torch.float32 else 2e-3)
    # the NCHW (VALU) path on the same level agrees
    nchw, = cc.forward(_t(f1, gpu, dtype), _t(f2, gpu, dtype), _t(co, gpu), _t(ii, gpu),
                       _t(jj, gpu), R)
    if dtype == torch.float32:
        _close(out.cpu().numpy(), nchw.cpu().numpy(), 1e-5)
    else:
        # fp16 features: both layouts accumulate the dot in fp32 (documented
        # deviation: the reference accumulates in fp16, correlation_kernel.cu:159)
        # and round once to the fp16 output; they differ only in the fp32
        # summation order, so the fp16 results agree to one fp16 ulp (2^-10
        # relative) of each value, plus 1e-6 of max|ref| for sums near zero
        a = out.double().cpu().numpy()
        b = nchw.double().cpu().numpy()
        tol = 2.0 ** -10 * np.abs(b) + 1e-6 * np.abs(b).max()
        assert (np.abs(a - b) <= tol).all(), np.abs(a - b).max()


def test_to_channels_last_frame_slot(gpu):
    from dpvo_amd import altcorr, synthetic

    src = torch.randn(1, 5, 128, 30, 40, device=gpu)
    dst = synthetic.channels_last(torch.zeros_like(src))
    altcorr.to_channels_last(src[0, 3], dst[0, 3])  # one frame of a ring buffer
    assert torch.equal(dst[0, 3], src[0, 3])
    assert torch.count_nonzero(dst[0, :3]) == 0
    full = altcorr.to_channels_last(src)
    assert torch.equal(full, src) and full.permute(0, 1, 3, 4, 2).is_contiguous()


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,scales", [(120, 160, (1, 2, 4, 8)), (120, 188, (1, 4)),
                                        (37, 45, (1, 2, 4, 8))])
def test_insert_frame_matches_avg_pool(gpu, H, W, scales):
    """One-launch pyramid insertion == avg_pool2d + channels-last copy, bit-exact,
    written only into the addressed ring slot (EuRoC 120x188 and ragged sizes)."""
    from dpvo_amd import altcorr, synthetic

    fmap = torch.randn(128, H, W, device=gpu)
    pyr = [synthetic.channels_last(torch.full((1, 4, 128, H // s, W // s), 7.0, device=gpu))
           for s in scales]
    altcorr.insert_frame(fmap, pyr, 2, scales)
    for p, s in zip(pyr, scales):
        ref = fmap if s == 1 else torch.nn.functional.avg_pool2d(fmap[None], s, s)[0]
        assert torch.equal(p[0, 2], ref), s
        assert bool((p[0, [0, 1, 3]] == 7.0).all())


def test_ordered_corr_matches_unordered(gpu):
    """XCD-aware edge order (reproject_ordered -> forward_levels(order=)):
    the order groups edges by target frame and is a permutation; the
    correlation is bit-identical to the unordered launch."""
    from dpvo_amd import altcorr, fastba, synthetic

    G = synthetic.make_config("cfg2", seed=5)
    D = G.to(gpu)
    mem = 36
    coords, order = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem)
    ref_c = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk)
    assert torch.equal(coords, ref_c)
    o = order.cpu().numpy()
    assert sorted(o.tolist()) == list(range(G.E))
    jj = G.jj.numpy()[o]
    assert (np.diff(jj) >= 0).all()  # grouped by target frame, groups in frame order
    # inside a frame: by the 16-pixel row band of the reprojected patch centre
    v = coords[0, :, 1, 1, 1].cpu().numpy()[o]
    band = np.where(v >= 0, np.minimum(v / 16.0, 15.0), 0).astype(np.int64)
    key = jj.astype(np.int64) * 16 + band
    assert (np.diff(key) >= 0).all()
    levels = (1, 2, 4, 8)
    pyr = [synthetic.channels_last(p) for p in
           synthetic.make_features(mem=mem, C=128, levels=levels, seed=1, device=gpu)]
    gmap = 0.25 * torch.randn(1, mem * G.M, 128, 3, 3, device=gpu)
    kk1, jj1 = D.kk % (mem * G.M), D.jj % mem
    a = altcorr.corr_levels(gmap, pyr, coords, kk1, jj1, 3, levels)
    b = altcorr.corr_levels(gmap, pyr, coords, kk1, jj1, 3, levels, order=order)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


# ---- fp16 features (MIXED_PRECISION): v_mfma_f32_16x16x16_f16 path ----
# fp16 x fp16 products are exact in fp32 and the MFMA accumulates in fp32, so
# against the fp64 oracle on the SAME fp16-rounded inputs only fp32 summation
# noise remains: |gpu - ref| <= 2e-5 * max(1, |ref|_max).  (The reference's
# fp16 path accumulates in fp16 -- an accuracy deviation in our favour.)
@pytest.mark.parametrize("kw", [dict(), dict(spread=4.0), dict(far=0.3),
                                dict(M=130, H2=12, W2=14)])
@pytest.mark.parametrize("levels", [(1,), (1, 4), (1, 2, 4, 8)])
def test_channels_last_fp16_matches_oracle(gpu, kw, levels):
    from dpvo_amd import altcorr, synthetic

    f1, f2, co, ii, jj, R = _case(13, **{**dict(M=67, C=128, H2=40, W2=48), **kw})
    f1h = _t(f1, gpu, torch.float16)
    lv1 = _t(f2, gpu, torch.float16)
    pyr = [lv1 if s == 1 else
           torch.nn.functional.avg_pool2d(lv1[0].float(), s, s).half().unsqueeze(0)
           for s in levels]
    out = altcorr.corr_levels(f1h, [synthetic.channels_last(p) for p in pyr], _t(co, gpu),
                              _t(ii, gpu), _t(jj, gpu), R, scales=levels)
    assert out.dtype == torch.float32
    out = out.view(1, len(ii), 2 * R + 1, 2 * R + 1, 3, 3, len(levels)).cpu().numpy()
    a = f1h.double().cpu().numpy()
    for l, s in enumerate(levels):
        ref = oracle.corr_fwd(a, pyr[l].double().cpu().numpy(), co / s, ii, jj, R)
        _close(out[..., l], ref, 2e-5)


def test_channels_last_fp16_equals_fp32_on_rounded_inputs(gpu):
    """The fp16 and fp32 matrix-core kernels agree on fp16-representable
    inputs at the full cfg2 edge count (only the K order differs)."""
    from dpvo_amd import altcorr, fastba, synthetic

    G = synthetic.make_config("cfg2", seed=6)
    D = G.to(gpu)
    mem, levels = 36, (1, 4)
    coords, order = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem)
    pyr = synthetic.make_features(mem=mem, C=128, levels=levels, seed=2, device=gpu)
    pyr16 = [synthetic.channels_last(p.half()) for p in pyr]
    pyr32 = [synthetic.channels_last(p.half().float()) for p in pyr]
    gmap = (0.25 * torch.randn(1, mem * G.M, 128, 3, 3, device=gpu)).half()
    kk1, jj1 = D.kk % (mem * G.M), D.jj % mem
    a = altcorr.corr_levels(gmap, pyr16, coords, kk1, jj1, 3, levels, order=order)
    b = altcorr.corr_levels(gmap.float(), pyr32, coords, kk1, jj1, 3, levels, order=order)
    torch.cuda.synchronize()
    err = (a - b).abs().max().item()
    assert err <= 1e-5 * max(1.0, b.abs().max().item()), err


@pytest.mark.parametrize("H,W,scales", [(120, 160, (1, 2, 4, 8)), (37, 45, (1, 2, 4, 8))])
def test_insert_frame_fp16(gpu, H, W, scales):
    """fp16 insertion: level 1 copied exactly, pooled levels = fp32 avg_pool2d
    of the halves rounded once to fp16 (torch's half avg_pool2d semantics)."""
    from dpvo_amd import altcorr, synthetic

    fmap = torch.randn(128, H, W, device=gpu).half()
    pyr = [synthetic.channels_last(torch.full((1, 3, 128, H // s, W // s), 7.0, device=gpu,
                                              dtype=torch.float16)) for s in scales]
    altcorr.insert_frame(fmap, pyr, 1, scales)
    for p, s in zip(pyr, scales):
        ref = fmap if s == 1 else torch.nn.functional.avg_pool2d(fmap[None].float(), s, s)[0].half()
        assert torch.equal(p[0, 1], ref), s
        assert bool((p[0, [0, 2]] == 7.0).all())


# ---- NCHW fp16 levels: matrix-core path (corr_nchw.hip) ----
# DPVO's own pyramid (dpvo.py:111-112: contiguous NCHW, fp16 under the default
# MIXED_PRECISION) through the unchanged per-level entry.  fp16 x fp16
# products are exact in fp32 and accumulate in fp32; the output is rounded
# once to fp16, so against the fp64 oracle on the same fp16 inputs each value
# is within one fp16 rounding (2^-11 relative, 2^-10 allowed) plus fp32
# summation noise (2e-5 of max|ref|).
def _close_f16(out, ref):
    out = np.asarray(out, np.float64)
    ref = np.asarray(ref, np.float64)
    assert out.shape == ref.shape
    tol = 2.0 ** -10 * np.abs(ref) + 2e-5 * max(1.0, np.abs(ref).max() if ref.size else 1.0)
    bad = np.abs(out - ref) > tol
    assert not bad.any(), (np.abs(out - ref).max(), int(bad.sum()))


def _f16_inputs(f1, f2):
    return f1.astype(np.float16), f2.astype(np.float16)


@pytest.mark.parametrize("kw", [
    dict(),                                   # W2 = 32: 16-B pieces
    dict(W2=36),                              # W2 % 8 == 4: 8-B pieces
    dict(W2=30, M=40),                        # W2 % 4 != 0: VALU kernel
    dict(R=0), dict(R=1), dict(R=2),
    dict(R=7),                                # box too wide for the image: raw path
    dict(p=1), dict(p=2), dict(p=4),
    dict(Hp=2, Wp=3),
    dict(spread=1.0, M=120),                  # image and raw edges mixed
    dict(spread=4.0),
    dict(far=0.5),                            # windows outside the map
    dict(B=2, M=11),
    dict(C=64, M=9),                          # C != 128: VALU kernel
    dict(H2=5, W2=8, M=21),                   # tiny map: every window clipped
    dict(M=300, H2=40, W2=48),
])
def test_nchw_fp16_forward_matches_oracle(cc, gpu, kw):
    f1, f2, co, ii, jj, R = _case(21, **kw)
    h1, h2 = _f16_inputs(f1, f2)
    out, = cc.forward(_t(h1, gpu), _t(h2, gpu), _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R)
    assert out.dtype == torch.float16
    ref = oracle.corr_fwd(h1.astype(np.float64), h2.astype(np.float64), co, ii, jj, R)
    _close_f16(out.cpu().numpy(), ref)


def test_nchw_fp16_unaligned_level_base(cc, gpu):
    """A level whose base is only 8-B aligned (a view at an odd offset) takes
    8-B pieces; a 2-B aligned one the VALU kernel: same results."""
    f1, f2, co, ii, jj, R = _case(22, M=90, H2=24, W2=32)
    h1, h2 = _f16_inputs(f1, f2)
    ref = oracle.corr_fwd(h1.astype(np.float64), h2.astype(np.float64), co, ii, jj, R)
    for shift in (4, 1):
        buf = torch.zeros(h2.size + shift, dtype=torch.float16, device=gpu)
        lv = buf[shift:].view(h2.shape)
        lv.copy_(_t(h2, gpu))
        out, = cc.forward(_t(h1, gpu), lv, _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R)
        _close_f16(out.cpu().numpy(), ref)


@pytest.mark.parametrize("levels", [(1, 4), (1, 2, 4, 8)])
def test_nchw_fp16_levels_match_oracle(gpu, levels):
    """corr_levels on an NCHW fp16 pyramid (float32 output): every level on
    the matrix-core kernel (W2 = 64, 32, 16, 8)."""
    from dpvo_amd import altcorr

    f1, f2, co, ii, jj, R = _case(23, M=150, C=128, H2=48, W2=64)
    h1, h2 = _f16_inputs(f1, f2)
    lv1 = _t(h2, gpu)
    pyr = [lv1 if s == 1 else
           torch.nn.functional.avg_pool2d(lv1[0].float(), s, s).half().unsqueeze(0).contiguous()
           for s in levels]
    out = altcorr.corr_levels(_t(h1, gpu), pyr, _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R,
                              scales=levels)
    out = out.view(1, len(ii), 2 * R + 1, 2 * R + 1, 3, 3, len(levels)).cpu().numpy()
    for l, s in enumerate(levels):
        ref = oracle.corr_fwd(h1.astype(np.float64), pyr[l].double().cpu().numpy(), co / s, ii,
                              jj, R)
        _close(out[..., l], ref, 2e-5)


def test_nchw_fp16_cfg2_matches_channels_last(cc, gpu):
    """The drop-in call at full cfg2 size (2048 edges, 36-frame fp16 ring,
    dpvo.py:462-465 verbatim) agrees with the channels-last kernel on the same
    data to one fp16 ulp, and with the oracle on a sample of edges."""
    from dpvo_amd import fastba, synthetic

    G = synthetic.make_config("cfg2", seed=7)
    D = G.to(gpu)
    mem, levels = 36, (1, 4)
    coords = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk)
    pyr = [p.half() for p in synthetic.make_features(mem=mem, C=128, levels=levels, seed=3,
                                                      device=gpu)]
    gmap = (0.25 * torch.randn(1, mem * G.M, 128, 3, 3, device=gpu)).half()
    kk1, jj1 = D.kk % (mem * G.M), D.jj % mem
    sel = np.arange(0, G.E, 37)
    for l, s in enumerate(levels):
        a, = cc.forward(gmap, pyr[l], coords / s, kk1, jj1, 3)
        b, = cc.forward(gmap, synthetic.channels_last(pyr[l]), coords / s, kk1, jj1, 3)
        a64, b64 = a.double().cpu().numpy(), b.double().cpu().numpy()
        tol = 2.0 ** -10 * np.abs(b64) + 1e-6 * np.abs(b64).max()
        assert (np.abs(a64 - b64) <= tol).all(), np.abs(a64 - b64).max()
        ref = oracle.corr_fwd(gmap.double().cpu().numpy(), pyr[l].double().cpu().numpy(),
                              (coords / s).cpu().numpy()[:, sel], kk1.cpu().numpy()[sel],
                              jj1.cpu().numpy()[sel], 3)
        _close_f16(a64[:, sel], ref)


# ---- NCHW fp32 levels: the same kernel with 16-channel images and
# v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 sums): the fp32 bar
@pytest.mark.parametrize("kw", [
    dict(),                                   # W2 = 32: 16-B pieces, 2 channels / load
    dict(W2=34, M=60),                        # W2 * 4 % 16 == 8: 8-B pieces
    dict(W2=36, spread=1.0, M=120),           # wide boxes: 1 channel / load, raw-path edges
    dict(R=1), dict(R=7), dict(p=2), dict(p=4), dict(Hp=2, Wp=3),
    dict(far=0.5), dict(B=2, M=11), dict(H2=5, W2=8, M=21),
    dict(M=300, H2=40, W2=48),
])
def test_nchw_fp32_forward_matches_oracle(cc, gpu, kw):
    f1, f2, co, ii, jj, R = _case(31, **kw)
    out, = cc.forward(_t(f1, gpu), _t(f2, gpu), _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R)
    assert out.dtype == torch.float32
    _close(out.cpu().numpy(), oracle.corr_fwd(f1, f2, co, ii, jj, R))


def test_nchw_fp32_cfg2_matches_channels_last(cc, gpu):
    """fp32 drop-in at full cfg2 size (36-frame ring, ordered path) against
    the channels-last kernel on the same data and the oracle on a sample."""
    from dpvo_amd import fastba, synthetic

    G = synthetic.make_config("cfg2", seed=8)
    D = G.to(gpu)
    mem, levels = 36, (1, 4)
    coords = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk)
    pyr = synthetic.make_features(mem=mem, C=128, levels=levels, seed=4, device=gpu)
    gmap = 0.25 * torch.randn(1, mem * G.M, 128, 3, 3, device=gpu)
    kk1, jj1 = D.kk % (mem * G.M), D.jj % mem
    sel = np.arange(0, G.E, 41)
    for l, s in enumerate(levels):
        a, = cc.forward(gmap, pyr[l], coords / s, kk1, jj1, 3)
        b, = cc.forward(gmap, synthetic.channels_last(pyr[l]), coords / s, kk1, jj1, 3)
        _close(a.cpu().numpy(), b.cpu().numpy(), 1e-5)
        ref = oracle.corr_fwd(gmap.cpu().numpy(), pyr[l].cpu().numpy(),
                              (coords / s).cpu().numpy()[:, sel], kk1.cpu().numpy()[sel],
                              jj1.cpu().numpy()[sel], 3)
        _close(a.cpu().numpy()[:, sel], ref)


# ---- fp32 features over a wide dynamic range: the
# channels-last fp32 path must hold the fp32 bar whatever the magnitudes
def _wide(seed, kind):
    f1, f2, co, ii, jj, R = _case(seed, M=96, C=128, H2=40, W2=48)
    r = np.random.default_rng(seed + 7)
    if kind == "channel_scales":  # per-channel scales 1e-4 .. 1e3 on both sides
        f1 = f1 * 10.0 ** r.uniform(-4, 3, (1, 1, 128, 1, 1))
        f2 = f2 * 10.0 ** r.uniform(-4, 3, (1, 1, 128, 1, 1))
    elif kind == "tiny":  # every feature ~1e-4 (f16-subnormal territory)
        f1, f2 = f1 * 1e-4, f2 * 1e-4
    elif kind == "large_a_tiny_b":
        f1, f2 = f1 * 1e3, f2 * 1e-4
    elif kind == "f16_edges":  # magnitudes at 2^-24, 2^-14, 2^-3, 1, 16
        e = r.choice([-24, -14, -3, 0, 4], size=f2.shape)
        f2 = np.sign(f2) * 2.0 ** e * (1 + 0.01 * r.standard_normal(f2.shape))
        e1 = r.choice([-14, -3, 0], size=f1.shape)
        f1 = np.sign(f1) * 2.0 ** e1 * (1 + 0.01 * r.standard_normal(f1.shape))
    elif kind == "beyond_f16":  # |b| >= 65520 in some pixels of the fine level
        m = r.random(f2.shape) < 0.02
        f2 = np.where(m, np.sign(f2) * r.uniform(65520, 3e5, f2.shape), f2)
    return f1.astype(np.float32), f2.astype(np.float32), co, ii, jj, R


@pytest.mark.parametrize("kind", ["channel_scales", "tiny", "large_a_tiny_b", "f16_edges",
                                  "beyond_f16"])
def test_channels_last_fp32_wide_range(gpu, kind):
    """Element-wise against the fp64 oracle: relative error <= 1e-4 wherever
    |ref| >= 1e-3 max|ref|, and everywhere |err| <= 1e-4 |ref| + 2^-20 S with
    S = the same correlation of |f1|, |f2| (the magnitude of the summed
    products: the fp32 summation-noise scale).  A plain sequential fp32 dot
    (the CUDA kernel's loop) measures 2.7e-5 .. 5.5e-5 on these cases under
    the first bar and needs 1.4e-8 .. 1.1e-7 S under the second."""
    from dpvo_amd import altcorr, synthetic

    f1, f2, co, ii, jj, R = _wide(41, kind)
    levels = (1, 4)
    lv1 = _t(f2, gpu)
    pyr = [lv1, torch.nn.functional.avg_pool2d(lv1[0], 4, 4).unsqueeze(0)]
    out = altcorr.corr_levels(_t(f1, gpu), [synthetic.channels_last(p) for p in pyr],
                              _t(co, gpu), _t(ii, gpu), _t(jj, gpu), R, scales=levels)
    out = out.view(1, len(ii), 2 * R + 1, 2 * R + 1, 3, 3, len(levels)).double().cpu().numpy()
    for l, s in enumerate(levels):
        p = pyr[l].cpu().numpy()
        ref = oracle.corr_fwd(f1, p, co / s, ii, jj, R).astype(np.float64)
        mag = oracle.corr_fwd(np.abs(f1), np.abs(p), co / s, ii, jj, R).astype(np.float64)
        err = np.abs(out[..., l] - ref)
        big = np.abs(ref) >= 1e-3 * np.abs(ref).max()
        rel = (err[big] / np.abs(ref[big])).max()
        assert rel <= 1e-4, (kind, s, rel)
        assert (err <= 1e-4 * np.abs(ref) + 2.0 ** -20 * mag).all(), (kind, s)
