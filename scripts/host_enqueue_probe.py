"""Where does the first step after a synchronize spend its host time?
(the driver's 20-step bench reads ~9 % below a long run;
bench.py's step_split showed the first timed step's enqueue at ~0.22 ms
against ~0.03 ms for the others.)

Builds bench.py's cfg2 step and times, with perf_counter and no sync, each
host call of a step -- frame-slot views, the fused reproject launch, A-CORR,
BA -- for (a) steady-state steps and (b) the first step after
torch.cuda.synchronize(), plus bare launches after a sync.  One JSON line.

    python scripts/host_enqueue_probe.py
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from dpvo_amd import altcorr, fastba, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    levels, mem = [1, 2, 4, 8], 36
    G = synthetic.make_config("cfg2", seed=0)
    D = G.to(dev)
    P, C = G.patches.shape[-1], 128
    pyr_nchw = synthetic.make_features(mem=mem, C=C, levels=levels, seed=0, device=dev)
    pyr = [synthetic.channels_last(p) for p in pyr_nchw]
    gbuf = torch.randn(1, mem * G.M, C, P, P, device=dev)
    lmbda = torch.tensor([1e-4], device=dev)
    poses, patches = D.poses.clone(), D.patches.clone()
    kk1, jj1 = D.kk % (G.M * mem), D.jj % mem
    scales = [float(s) for s in levels]

    def step(i, t=None):
        slot = i % mem
        a = time.perf_counter()
        dst = [p[0, slot] for p in pyr]
        b = time.perf_counter()
        coords, order, ws = fastba.reproject(poses, patches, D.intrinsics, D.ii, D.jj, D.kk,
                                             mem=mem, plan_window=(1, G.F),
                                             insert=(pyr_nchw[0][0, slot], dst, levels))
        c = time.perf_counter()
        altcorr.corr_levels(gbuf, pyr, coords, kk1, jj1, 3, scales, order=order)
        d = time.perf_counter()
        fastba.BA(poses, patches, D.intrinsics, D.target, D.weight, lmbda, D.ii, D.jj, D.kk, 1,
                  G.F, M=G.M, iterations=2, plan=ws)
        e = time.perf_counter()
        if t is not None:
            t.append([b - a, c - b, d - c, e - d])

    for i in range(300):
        step(i)
    torch.cuda.synchronize()
    names = ["views", "reproject+plan+insert", "corr", "BA"]
    steady = []
    for i in range(200):
        step(i, steady)
    torch.cuda.synchronize()
    first = []
    for i in range(30):
        torch.cuda.synchronize()
        time.sleep(0.002)
        step(i, first)
    torch.cuda.synchronize()
    # the same after a sync but with no idle gap
    first_nosleep = []
    for i in range(30):
        torch.cuda.synchronize()
        step(i, first_nosleep)
    torch.cuda.synchronize()
    # a bare launch after a sync (runtime wake-up?)
    x = torch.zeros(16, device=dev)
    bare = []
    for i in range(30):
        torch.cuda.synchronize()
        a = time.perf_counter()
        x.add_(1.0)
        bare.append(time.perf_counter() - a)
    steady_bare = []
    for i in range(30):
        a = time.perf_counter()
        x.add_(1.0)
        steady_bare.append(time.perf_counter() - a)
    torch.cuda.synchronize()

    def med(rows):
        cols = list(zip(*rows))
        return {n: round(1e6 * sorted(c)[len(c) // 2], 1) for n, c in zip(names, cols)}

    out = {"unit": "us (host, median)", "steady": med(steady),
           "first_after_sync_idle2ms": med(first), "first_after_sync": med(first_nosleep),
           "bare_launch_after_sync": round(1e6 * sorted(bare)[15], 1),
           "bare_launch_steady": round(1e6 * sorted(steady_bare)[15], 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
