"""Autograd wrappers over the `cuda_corr` extension (A-CORR, A-CORR-BWD,
A-PATCH, A-PATCH-BWD).

Reference surface: dpvo/altcorr/correlation.py:14-84 (cuteboyqq/DPVO).
  * corr(fmap1, fmap2, coords, ii, jj, radius=1, dropout=1)
        -> [B, M, 2R+1, 2R+1, p, p], the bilinear-interpolated correlation of
           gmap patch ii[m] against frame jj[m] around coords (correlation.py:83-84).
           The fork's runtime evaluated this with a Python fp16 grid_sample
           (correlation_kernel.py:552-654); here it is the HIP kernel with fp32
           accumulation for every input dtype (output in the input dtype).
  * patchify(net, coords, radius, mode='bilinear') (correlation.py:63-80).
           `BORDER_MODE` selects the border rule of the gather: "clamp" (default,
           the fork's runtime patchify_forward_kernel_python,
           correlation_kernel.py:181-224) or "zero" (the CUDA kernel,
           correlation_kernel.cu:16-47).  Backward uses the same rule.
"""
from __future__ import annotations

import torch

from .._native import load_extension, require_gpu

cuda_corr = load_extension("cuda_corr")

BORDER_MODE = "clamp"


class CorrLayer(torch.autograd.Function):
    """correlation.py:14-41."""

    @staticmethod
    def forward(ctx, fmap1, fmap2, coords, ii, jj, radius, dropout):
        require_gpu(fmap1)
        ctx.save_for_backward(fmap1, fmap2, coords, ii, jj)
        ctx.radius = radius
        ctx.dropout = dropout
        out, = cuda_corr.forward(fmap1, fmap2, coords, ii, jj, radius)
        return out

    @staticmethod
    def backward(ctx, grad):
        fmap1, fmap2, coords, ii, jj = ctx.saved_tensors
        if ctx.dropout < 1:  # edge dropout of the training path (correlation.py:31-36)
            keep = torch.rand(len(ii), device=grad.device) < ctx.dropout
            coords, grad, ii, jj = coords[:, keep], grad[:, keep], ii[keep], jj[keep]
        g1, g2 = cuda_corr.backward(fmap1, fmap2, coords, ii, jj, grad.contiguous(), ctx.radius)
        return g1, g2, None, None, None, None, None


class PatchLayer(torch.autograd.Function):
    """correlation.py:44-61 (border rule: BORDER_MODE)."""

    @staticmethod
    def forward(ctx, net, coords, radius):
        require_gpu(net)
        ctx.radius = radius
        ctx.clamp = BORDER_MODE == "clamp"
        ctx.save_for_backward(net, coords)
        fn = cuda_corr.patchify_forward_clamped if ctx.clamp else cuda_corr.patchify_forward
        patches, = fn(net, coords, radius)
        return patches

    @staticmethod
    def backward(ctx, grad):
        net, coords = ctx.saved_tensors
        fn = cuda_corr.patchify_backward_clamped if ctx.clamp else cuda_corr.patchify_backward
        g, = fn(net, coords, grad.contiguous(), ctx.radius)
        return g, None, None


def patchify(net, coords, radius, mode="bilinear"):
    """Extract (2R+2)^2 windows; with mode='bilinear' resample them to (2R+1)^2
    at the fractional offset of each centre (correlation.py:63-80)."""
    patches = PatchLayer.apply(net, coords, radius)
    if mode != "bilinear":
        return patches
    frac = coords - coords.floor()
    dx = frac[..., 0][:, :, None, None, None]
    dy = frac[..., 1][:, :, None, None, None]
    d = 2 * radius + 1
    # same term order as correlation.py:74-80 (bit-identical in fp32)
    w = ((1 - dy) * (1 - dx), (1 - dy) * dx, dy * (1 - dx), dy * dx)
    win = (patches[..., :d, :d], patches[..., :d, 1:], patches[..., 1:, :d], patches[..., 1:, 1:])
    return w[0] * win[0] + w[1] * win[1] + w[2] * win[2] + w[3] * win[3]


def corr(fmap1, fmap2, coords, ii, jj, radius=1, dropout=1):
    """correlation.py:83-84."""
    return CorrLayer.apply(fmap1, fmap2, coords, ii, jj, radius, dropout)


def to_channels_last(src, dst=None):
    """Copy a [..., C, H, W] feature map into channels-last memory (HIP
    transpose); ``dst`` (same shape, channels-last) is filled in place, e.g.
    one frame slot of a channels-last pyramid ring buffer."""
    require_gpu(src)
    if dst is None:
        perm = list(range(src.dim() - 3)) + [src.dim() - 2, src.dim() - 1, src.dim() - 3]
        inv = [perm.index(i) for i in range(src.dim())]
        dst = src.new_empty([src.shape[i] for i in perm]).permute(inv)
    cuda_corr.feature_to_nhwc(src, dst)
    return dst


def insert_frame(fmap, pyramid, slot, scales=(1, 4)):
    """Write one new frame into a channels-last pyramid ring buffer in ONE
    launch: level s of ring slot ``slot`` = avg_pool2d(fmap, s, s) (level 1 =
    fmap itself), the frame insertion of dpvo.py (fmap1_/fmap2_ ring writes,
    dpvo.py:462-463 read them back).  ``fmap`` is the NCHW [C, H, W] level-1
    frame; ``pyramid[l]`` are [B, mem, C, H/s, W/s] channels-last buffers."""
    require_gpu(fmap)
    cuda_corr.feature_pyramid_insert(fmap, [p[0, slot] for p in pyramid],
                                     [int(s) for s in scales])


def insert_frame_ring(fmap, pyramid, slot_dev, scales=(1, 4)):
    """insert_frame with the ring slot read on the device: slot = slot_dev[0] %
    mem (int32 device scalar), so a captured update graph can be replayed for
    every new frame."""
    require_gpu(fmap)
    cuda_corr.feature_pyramid_insert_ring(fmap, list(pyramid), [int(s) for s in scales], slot_dev)


def corr_levels(fmap1, pyramid, coords, ii, jj, radius=3, scales=(1, 4), order=None):
    """DPVO.corr (dpvo/dpvo.py:456-465) in ONE launch: correlation of every
    pyramid level (coords divided by each level's scale) stacked on the last
    axis and flattened to [B, M, (2R+1)^2 * p^2 * L] float32.  Inference only.

    Levels stored channels-last (``synthetic.channels_last`` / ``to_channels_last``)
    take the matrix-core path (corr_nhwc.hip); NCHW levels the VALU path.
    float16 features (the fork's MIXED_PRECISION runtime) run on
    v_mfma_f32_16x16x16_f16 with fp32 accumulation; the output stays float32.
    ``order`` (int32 [E], from ``fastba.reproject(..., mem=N2)``): process
    edges grouped by target frame, one group range per XCD (same results)."""
    require_gpu(fmap1)
    out = cuda_corr.forward_levels(fmap1, list(pyramid), coords, ii, jj, radius,
                                   [float(s) for s in scales], order)
    return out.view(out.shape[0], out.shape[1], -1)
