"""Why does the update harness's window pose error grow with the patch count
M (0.011 m scaled at M = 10, 0.042 m at M = 20)?  Runs
the harness (eager, 80 frames) over M, the oracle network's perturbation
amplitude (0 = exact targets) and the BA iteration count, and reports the
scaled / unscaled window pose error, the scale and the depth error.

    python scripts/harness_error_study.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from dpvo_amd.update import UpdateHarness  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 80
for iters in (1, 2):
    for noise in (0.0, 0.1):
        for M in (5, 10, 15, 20):
            h = UpdateHarness(M=M, ba_iters=iters, buffer=frames + 8, net_noise=noise)
            errs = []
            for f in range(frames):
                h.step()
                if f >= 20 and f % 10 == 9:
                    errs.append(round(h.pose_error_scaled()[0], 4))
            err, scale = h.pose_error_scaled()
            print(json.dumps({"M": M, "net_noise": noise, "ba_iters": iters, "frames": frames,
                              "edges": h.pg.num_edges, "pose_err_m": h.pose_error(),
                              "pose_err_scaled_m": err, "scale": scale,
                              "scaled_err_by_frame": errs,
                              "depth_err": h.depth_error(h.n - 20, h.n - 12),
                              "status": h.check()}), flush=True)
            del h
            torch.cuda.empty_cache()
