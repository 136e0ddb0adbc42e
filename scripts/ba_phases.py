"""Per-phase timing of the fused F-BA kernel on cfg2 (GPU): wall-clock marks
stamped by thread 0 after every phase (cuda_ba.forward_marks)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dpvo_amd  # noqa: E402
from dpvo_amd import synthetic  # noqa: E402

cb = dpvo_amd.load_extension("cuda_ba")
dev = torch.device("cuda:0")
cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
G = synthetic.make_config(cfg, seed=0)
D = G.to(dev)
lm = torch.tensor([1e-4], device=dev)
names = ["linearize", "patch", "schur", "solve", "update"]
acc = {}
for rep in range(20):
    poses, patches = D.poses.clone(), D.patches.clone()
    m = cb.forward_marks(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk,
                         G.M, 1, G.F, iters, False).cpu().tolist()
    if rep < 5:
        continue
    d = {"setup": m[1] - m[0]}
    prev = m[1]
    for it in range(iters):
        for k, n in enumerate(names):
            t = m[2 + 5 * it + k]
            d[f"{n}{it}"] = t - prev
            prev = t
    d["total"] = prev - m[0]
    for k, v in d.items():
        acc.setdefault(k, []).append(v * 10.0 / 1000.0)  # 100 MHz ticks -> us
for k, v in acc.items():
    v.sort()
    print(f"{k:12s} median {v[len(v) // 2]:8.2f} us")
