"""Per-frame timing of DPVO's update data flow on the MI355X ops
(dpvo_amd/update.py: insertion, device patch graph, reproject + plan, corr
levels [1,4], deterministic oracle network, fastba.BA window, keyframe-window
removal), eager and as replayed hipGraphs, plus the window pose error before
and after a global scale (monocular BA fixes the scene only up to scale).

    python scripts/dpvo_update_bench.py [frames=80] [M=20] [ba_iters=1]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from dpvo_amd.update import UpdateHarness  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 80
M = int(sys.argv[2]) if len(sys.argv) > 2 else 20
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1
h = UpdateHarness(M=M, ba_iters=iters, buffer=frames + 8)
warm = 40
for f in range(warm):
    st = h.step()
eager = [s["total_ms"] for s in h.stats[-10:]]
h.capture()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
h.replay(frames - warm)
ev[1].record()
torch.cuda.synchronize()
per = ev[0].elapsed_time(ev[1]) / (frames - warm)
err, scale = h.pose_error_scaled()
print(json.dumps({"M": M, "edges": st["edges"], "ba_iters": iters, "frames": frames,
                  "eager_ms_per_frame_median": sorted(eager)[len(eager) // 2],
                  "graph_ms_per_frame": per, "pose_err_m": h.pose_error(),
                  "pose_err_scaled_m": err, "scale": scale,
                  "depth_err": h.depth_error(h.n - 20, h.n - 12), "status": h.check()}))
