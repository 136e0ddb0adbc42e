"""A-CORR through the reference's own per-level entry (cuda_corr.forward,
dpvo.py:462-465: one call per level, then torch.stack) on DPVO's pyramid
layout -- contiguous NCHW rings (dpvo.py:111-112), fp32 and fp16
(MIXED_PRECISION) -- against the fused channels-last launch the bench times,
cfg2 (2048 edges, mem 36).  HIP-event medians per call, one JSON line per
variant.

    python scripts/corr_dropin_bench.py [--reps 50]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import dpvo_amd._native as _nat  # noqa: E402

if "--native" in sys.argv:  # A/B: extension modules from another build directory
    _nat.NATIVE_DIR = os.path.abspath(sys.argv[sys.argv.index("--native") + 1])

from dpvo_amd import altcorr, fastba, synthetic  # noqa: E402


def timed(fn, reps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--native", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    from dpvo_amd.altcorr.correlation import cuda_corr as cc
    G = synthetic.make_config("cfg2", seed=0)
    D = G.to(dev)
    mem, R = 36, 3
    coords = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk)
    kk1, jj1 = D.kk % (G.M * mem), D.jj % mem
    for levels in ((1, 4), (1, 2, 4, 8)):
        for dt in (torch.float32, torch.float16):
            pyr = synthetic.make_features(mem=mem, C=128, levels=levels, seed=0, device=dev, dtype=dt)
            gmap = (0.25 * torch.randn(1, mem * G.M, 128, 3, 3, device=dev)).to(dt)
            pcl = [synthetic.channels_last(p) for p in pyr]
            sc = [float(s) for s in levels]

            def dpvo_calls(p=pyr):  # dpvo.py:462-465 verbatim: per level, then stack
                return torch.stack([cc.forward(gmap, p[l], coords / s, kk1, jj1, R)[0]
                                    for l, s in enumerate(sc)], -1)

            rows = {
                "per_level_forward_nchw": lambda: dpvo_calls(pyr),
                "per_level_forward_channels_last": lambda: dpvo_calls(pcl),
                "forward_levels_nchw": lambda: altcorr.corr_levels(gmap, pyr, coords, kk1, jj1, R,
                                                                   sc),
                "forward_levels_channels_last": lambda: altcorr.corr_levels(gmap, pcl, coords, kk1,
                                                                            jj1, R, sc),
            }
            base = None
            for name, fn in rows.items():
                us = timed(fn, args.reps)
                base = us if name == "forward_levels_channels_last" else base
                print(json.dumps({"variant": name, "levels": list(levels),
                                  "dtype": str(dt).split(".")[-1], "edges": G.E, "us": us}),
                      flush=True)
            del pyr, pcl


if __name__ == "__main__":
    main()
