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
                       ("setup -> solve tail", 42, 49), ("solve.factor0", 49, 50),
                       ("solve.factorise", 50, 51), ("solve.substitute", 51, 52)]:
        d[name] = (m[b] - m[a]) * 10.0 / 1000.0
    wg = m[64:]
    NL = (G.F - 1) * G.F // 2
    starts, ends = wg[0::2], wg[1::2]
    t0 = min(starts)
    dur = [(e - s) * 0.01 for s, e in zip(starts, ends)]
    d["iter: first WG start -> last WG end"] = (max(ends) - t0) * 0.01
    d["iter: diag WG max dur"] = max(dur[i] for i in range(NL)
                                     if i == (int((8 * i + 1) ** 0.5 - 1) // 2) *
                                     ((int((8 * i + 1) ** 0.5 - 1) // 2) + 3) // 2)
    d["iter: off WG max dur"] = max(dur[:NL])
    d["iter: owner WG max dur"] = max(dur[NL:])
    d["iter: WG start spread"] = (max(starts) - t0) * 0.01
    for k, v in d.items():
        acc.setdefault(k, []).append(v)
for k, v in acc.items():
    v.sort()
    print(f"{k:22s} median {v[len(v) // 2]:8.2f} us")
