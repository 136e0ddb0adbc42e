"""The fork's live local BA call (dpvo.py:818-824: one iteration over the
optimisation window, t0 = n - 10) on a DPVO-pattern window
(synthetic.make_dpvo_window, M = 25 -> E = 9850, N = 10), as DPVO issues it:
cuda_ba.forward with no plan, so the call is the plan launch + the window
kernel.  HIP-event median per call over --reps calls; run it under
`rocprofv3 --kernel-trace --stats` (scripts/gpu.sh dpvoprof) for the
per-kernel split.

    python scripts/dpvo_window_call.py [--M 25] [--iters 1] [--reps 300]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dpvo_amd  # noqa: E402
from dpvo_amd import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=25)
    ap.add_argument("--iters", type=int, default=1)
    ap.add_argument("--reps", type=int, default=300)
    args = ap.parse_args()
    cb = dpvo_amd.load_extension("cuda_ba")
    dev = torch.device("cuda:0")
    lm = torch.tensor([1e-4], device=dev)
    G = synthetic.make_dpvo_window(M=args.M, seed=args.M)
    D = G.to(dev)
    t0, t1 = G.F - 10, G.F
    poses, patches = D.poses.clone(), D.patches.clone()

    def call():
        poses.copy_(D.poses)
        patches.copy_(D.patches)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        cb.forward(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, G.M,
                   t0, t1, args.iters, False)
        ev[1].record()
        return ev

    for _ in range(30):
        call()
    torch.cuda.synchronize()
    evs = [call() for _ in range(args.reps)]
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
    cb.check_status(poses)
    print(json.dumps({"graph": f"dpvo window M={args.M}", "E": G.E, "N": t1 - t0,
                      "iterations": args.iters, "call_us_median": round(ts[len(ts) // 2], 2),
                      "call_us_min": round(ts[0], 2), "reps": args.reps}))


if __name__ == "__main__":
    main()
