"""Per-phase timing of the F-BA kernels from the wall-clock stamps (100 MHz)
they leave in the workspace.  path 0/3 = per-block workgroups (ba_blocks.hip):
  [0] start, [1] setup done, per iteration (base 2 + 8 it): +0 workgroup 0's
  block assembled, +1 every block arrived, +2 solve done; [63] end.
path 1 = single workgroup (ba_fused.hip): per iteration +0 E phase, +1 B/Schur
assembly, +2 solve + poses, +3 inverse depths.

    python scripts/ba_fused_phases.py [cfg] [iterations] [path]
"""
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
path = int(sys.argv[3]) if len(sys.argv) > 3 else 0
cb.select_path(path)
names = (["E (patch sums)", "B+Schur assembly", "solve+poses", "depths"] if path == 1 else
         ["WG0 patch loop", "WG0 reduce+store", "all blocks arrived", "gather S",
          "forward elimination", "back substitution", "publish dX"])
G = synthetic.make_config(cfg, seed=0)
D = G.to(dev)
lm = torch.tensor([1e-4], device=dev)
acc = {}
for rep in range(40):
    poses, patches = D.poses.clone(), D.patches.clone()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cb.forward(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, G.M, 1,
               G.F, iters, False)
    e1.record()
    torch.cuda.synchronize()
    m = cb.forward_marks(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk,
                         G.M, 1, G.F, iters, False).cpu().tolist()
    if rep < 5:
        continue
    d = {"call (events)": e0.elapsed_time(e1) * 1e3, "kernel (stamps)": (m[63] - m[0]) * 0.01,
         "setup": (m[1] - m[0]) * 0.01}
    if path != 1:
        d["setup.loads"] = (m[40] - m[0]) * 0.01
        d["setup.sort"] = (m[41] - m[40]) * 0.01
        d["setup.relevant"] = (m[42] - m[41]) * 0.01
        d["setup.tables"] = (m[1] - m[42]) * 0.01
    prev = m[1]
    for it in range(iters):
        b = 2 + 8 * it
        for k, name in enumerate(names):
            d[f"it{it}.{name}"] = (m[b + k] - prev) * 0.01
            prev = m[b + k]
    d["tail (update + write-back)"] = (m[63] - prev) * 0.01
    for k, v in d.items():
        acc.setdefault(k, []).append(v)
for k, v in acc.items():
    v.sort()
    print(f"{k:26s} median {v[len(v) // 2]:8.2f} us")
