"""Timing of one F-BA call (GPU): CUDA-event total per call, plus the
wall-clock stamps the kernels leave in the workspace (cuda_ba.forward_marks):
setup start/sort/end, and in iteration 0 the solve tail (start, first
factor, factorisation, substitution).

    python scripts/ba_phases.py [cfg] [iterations]
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
G = synthetic.make_config(cfg, seed=0)
D = G.to(dev)
lm = torch.tensor([1e-4], device=dev)
acc = {}
for rep in range(30):
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
    d = {"call (events)": e0.elapsed_time(e1) * 1e3}
    for name, a, b in [("setup.sort", 40, 41), ("setup.masks", 41, 42),
                       ("setup end -> solve tail", 42, 49), ("tail: load + inv0", 49, 50),
                       ("tail: gauss-jordan", 50, 51), ("tail: update", 51, 52)]:
        d[name] = (m[b] - m[a]) * 10.0 / 1000.0
    N = G.F - 1
    for k in range(N):
        d[f"gj.k{k:02d}.pivot"] = (m[60 + 2 * k] - (m[50] if k == 0 else m[59 + 2 * k])) * 0.01
        d[f"gj.k{k:02d}.elim"] = (m[61 + 2 * k] - m[60 + 2 * k]) * 0.01
    for nm, base in [("WG0", 100), ("WGlast", 105)]:
        d[f"{nm}.compact"] = (m[base] - m[128 + 2 * (0 if nm == 'WG0' else (N * (N + 1) // 2 - 1))]) * 0.01
        d[f"{nm}.gather"] = (m[base + 1] - m[base]) * 0.01
        d[f"{nm}.sum"] = (m[base + 2] - m[base + 1]) * 0.01
    wg = m[128:]
    NL = (G.F - 1) * G.F // 2
    starts, ends = wg[0::2], wg[1::2]
    t0 = min(starts)
    dur = [(e - s) * 0.01 for s, e in zip(starts, ends)]
    d["iter: first WG start -> last WG end"] = (max(ends) - t0) * 0.01
    d["iter: Schur WG max dur"] = max(dur)
    d["iter: Schur WG min dur"] = min(dur)
    d["iter: WG start spread"] = (max(starts) - t0) * 0.01
    for k, v in d.items():
        acc.setdefault(k, []).append(v)
for k, v in acc.items():
    v.sort()
    print(f"{k:22s} median {v[len(v) // 2]:8.2f} us")
