"""Where does the NCHW fp16 matrix-core corr (corr_nchw.hip) spend its time?
Times one per-level cuda_corr.forward at cfg2 (level 1 and level 4, fp16
NCHW ring of 36 frames) for the same edges presented in different orders:
  given      the synthetic graph's edge order
  sorted     edges sorted by target frame (a frame's edges on consecutive
             workgroups, i.e. spread over all 8 XCDs round-robin)
  xcd        sorted by target frame and dealt so that XCD x (workgroup w
             runs on XCD w % 8) gets the x-th eighth of the sorted edges
  oneframe   every edge aimed at frame 0 (upper bound on L2 reuse)
HIP-event medians per call.  python scripts/nchw_order_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from dpvo_amd import fastba, synthetic  # noqa: E402


def timed(fn, reps=40):
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
    dev = torch.device("cuda:0")
    from dpvo_amd.altcorr.correlation import cuda_corr as cc
    G = synthetic.make_config("cfg2", seed=0)
    D = G.to(dev)
    mem, R = 36, 3
    coords = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk)
    kk1, jj1 = D.kk % (G.M * mem), D.jj % mem
    E = len(jj1)
    srt = torch.argsort(jj1 * E + torch.arange(E, device=dev))
    # XCD deal: workgroup w (4 edges) runs on XCD w % 8; XCD x takes sorted chunk x
    nwg = (E + 3) // 4
    per = (nwg + 7) // 8
    pos = []
    for w in range(nwg):
        chunk = (w % 8) * per + w // 8
        pos.extend(range(4 * chunk, min(4 * chunk + 4, E)) if chunk < nwg else [])
    xcd = srt[torch.tensor([p for p in pos if p < E], device=dev)]
    orders = {"given": torch.arange(E, device=dev), "sorted": srt, "xcd": xcd}
    for s, lvl in ((1, 0), (4, 1)):
        pyr = synthetic.make_features(mem=mem, C=128, levels=(1, 4), seed=0, device=dev,
                                      dtype=torch.float16)
        gmap = (0.25 * torch.randn(1, mem * G.M, 128, 3, 3, device=dev)).half()
        f2 = pyr[lvl]
        co = coords / s
        for name, o in orders.items():
            c, k, j = co[:, o].contiguous(), kk1[o].contiguous(), jj1[o].contiguous()
            us = timed(lambda: cc.forward(gmap, f2, c, k, j, R))
            print(json.dumps({"level": s, "order": name, "us": round(us, 2)}), flush=True)
        j0 = torch.zeros_like(jj1)
        us = timed(lambda: cc.forward(gmap, f2, co, kk1, j0, R))
        print(json.dumps({"level": s, "order": "oneframe", "us": round(us, 2)}), flush=True)
        cl = synthetic.channels_last(f2)
        us = timed(lambda: cc.forward(gmap, cl, co, kk1, jj1, R))
        print(json.dumps({"level": s, "order": "channels_last_given", "us": round(us, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
