"""Kernel-level profile target for the drop-in NCHW fp16 per-level call
(dpvo.py:462-465 verbatim: cuda_corr.forward per level, then torch.stack) at
cfg2, against the same call on channels-last levels.  Run under
rocprofv3 --kernel-trace --stats; prints HIP-event medians too.
    python scripts/corr_nchw_prof.py [--reps 100]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from dpvo_amd import fastba, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    from dpvo_amd.altcorr.correlation import cuda_corr as cc
    G = synthetic.make_config("cfg2", seed=0)
    D = G.to(dev)
    mem, R, levels = 36, 3, (1, 4)
    coords = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk)
    kk1, jj1 = D.kk % (G.M * mem), D.jj % mem
    pyr = synthetic.make_features(mem=mem, C=128, levels=levels, seed=0, device=dev,
                                  dtype=torch.float16)
    pcl = [synthetic.channels_last(p) for p in pyr]
    gmap = (0.25 * torch.randn(1, mem * G.M, 128, 3, 3, device=dev)).half()

    def dpvo_calls(p):  # dpvo.py:462-465
        return torch.stack([cc.forward(gmap, p[l], coords / s, kk1, jj1, R)[0]
                            for l, s in enumerate(levels)], -1)

    for name, p in (("nchw", pyr), ("channels_last", pcl)):
        for _ in range(10):
            dpvo_calls(p)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            dpvo_calls(p)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        ts.sort()
        print(json.dumps({"layout": name, "levels": list(levels), "dtype": "float16",
                          "edges": G.E, "us_median": round(ts[len(ts) // 2], 2)}), flush=True)


if __name__ == "__main__":
    main()
