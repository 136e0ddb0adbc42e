"""Per-frame timing of DPVO's update data flow on the MI355X ops
(dpvo_amd/update.py: insertion, device patch graph, reproject, corr levels
[1,4], synthetic oracle network, fastba.BA window, keyframe-window removal).

    python scripts/dpvo_update_bench.py [frames=60] [M=96] [ba_iters=2] [fp16]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from dpvo_amd import fastba  # noqa: E402
from dpvo_amd.update import UpdateHarness  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 60
M = int(sys.argv[2]) if len(sys.argv) > 2 else 96
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 2
dt = torch.float16 if (len(sys.argv) > 4 and sys.argv[4] == "fp16") else torch.float32
h = UpdateHarness(M=M, ba_iters=iters, feat_dtype=dt)
for f in range(frames):
    st = h.step()
    if f % 10 == 0 or f == frames - 1:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()}),
              flush=True)
tail = h.stats[frames // 2:]
keys = [k for k in tail[0] if k.endswith("_ms")]
med = {k: sorted(s[k] for s in tail)[len(tail) // 2] for k in keys}
print(json.dumps({"summary": f"median of the last {len(tail)} frames", "M": M, "ba_iters": iters,
                  "features": str(dt), "edges": tail[-1]["edges"], **med,
                  "pose_err_m": h.pose_error(),
                  "ba_status": fastba.cuda_ba.check_status(h.poses)}), flush=True)
