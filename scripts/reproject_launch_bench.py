"""Where the time of the update's first launch goes:
HIP-event medians at cfg2 (and a DPVO window) of the fused frame insertion +
reprojection + A-CORR edge order + BA plan launch against its parts run
alone -- reproject (+ order), the plan kernel, the pyramid insertion.

    python scripts/reproject_launch_bench.py [cfg2|dpvo25 ...]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from dpvo_amd import altcorr, fastba, synthetic  # noqa: E402


def timed(fn, reps=60):
    for _ in range(10):
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
    mem, levels = 36, (1, 2, 4, 8)
    pyr_nchw = synthetic.make_features(mem=mem, C=128, levels=levels, seed=0, device=dev)
    pyr = [synthetic.channels_last(p) for p in pyr_nchw]
    for name in (sys.argv[1:] or ["cfg2", "dpvo25"]):
        if name == "cfg2":
            G = synthetic.make_config("cfg2", seed=0)
            t0, t1 = 1, G.F
        else:
            G = synthetic.make_dpvo_window(M=25, seed=25)
            t0, t1 = G.F - 10, G.F
        D = G.to(dev)
        ins = (pyr_nchw[0][0, 3], [p[0, 3] for p in pyr], levels)
        rows = {
            "fused: insert + reproject + order + plan": lambda: fastba.reproject(
                D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem,
                plan_window=(t0, t1), insert=ins),
            "reproject + order + plan": lambda: fastba.reproject(
                D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem, plan_window=(t0, t1)),
            "reproject + order": lambda: fastba.reproject(
                D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem),
            "reproject": lambda: fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj,
                                                  D.kk),
            "plan kernel": lambda: fastba.plan(D.ii, D.jj, D.kk, t0, t1, D.patches.shape[0],
                                               D.poses.shape[0]),
            "pyramid insertion": lambda: altcorr.insert_frame(pyr_nchw[0][0, 3], pyr, 3, levels),
        }
        for k, fn in rows.items():
            print(json.dumps({"graph": name, "E": G.E, "launch": k, "us": timed(fn)}), flush=True)


if __name__ == "__main__":
    main()
