"""F-BA latency per cuda_ba.forward call (HIP events, median of 50) on the
bench graph (cfg2) and on DPVO-pattern local windows (make_dpvo_window:
M = 10 / 18 / 25 -> E ~ 4k / 7k / 10k, N = 10 free poses, t0 = n - 10),
iterations 1 (the fork's local call, dpvo.py:824) and 2 (fastba default).

    python scripts/ba_window_bench.py > profiles/rNN_ba_window.txt
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dpvo_amd  # noqa: E402
from dpvo_amd import synthetic  # noqa: E402

cb = dpvo_amd.load_extension("cuda_ba")
dev = torch.device("cuda:0")
lm = torch.tensor([1e-4], device=dev)
cases = [("cfg2 (bench graph)", synthetic.make_config("cfg2", seed=0), 1, 12)]
for M in (10, 18, 25):
    G = synthetic.make_dpvo_window(M=M, seed=M)
    cases.append((f"dpvo window M={M}", G, G.F - 10, G.F))
print(f"{'graph':22s} {'E':>6s} {'N':>3s} {'iters':>5s} {'us/call':>9s}")
for name, G, t0, t1 in cases:
    D = G.to(dev)
    for iters in (1, 2):
        ts = []
        for rep in range(60):
            poses, patches = D.poses.clone(), D.patches.clone()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            cb.forward(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, G.M,
                       t0, t1, iters, False)
            b.record()
            torch.cuda.synchronize()
            if rep >= 10:
                ts.append(a.elapsed_time(b) * 1e3)
        ts.sort()
        print(f"{name:22s} {G.E:6d} {t1 - t0:3d} {iters:5d} {ts[len(ts) // 2]:9.1f}", flush=True)
st = cb.check_status(D.poses)
print("status", st)
