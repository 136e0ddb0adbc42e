"""Timing of cuda_ba.solve_system (Sim3 pose graph, ba.cpp:120-180) on the
device: n poses, odometry chain + random loop edges (tests/test_pgo.py
generator), median of HIP-event timings of the whole call (assembly kernels +
fp64 Cholesky + host index checks)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dpvo_amd  # noqa: E402
from test_pgo import make_pgo  # noqa: E402

cb = dpvo_amd.load_extension("cuda_ba")
dev = torch.device("cuda:0")
for n, r in [(100, 300), (500, 1500), (1000, 3000), (2000, 6000)]:
    Ji, Jj, ii, jj, res = [torch.from_numpy(a).to(dev) for a in make_pgo(n, r, seed=0)]
    for _ in range(3):
        cb.solve_system(Ji, Jj, ii, jj, res, 1e-4, 1e-4, n - 1)
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        cb.solve_system(Ji, Jj, ii, jj, res, 1e-4, 1e-4, n - 1)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    print(f"solve_system n={n} r={r}: {sorted(ts)[5]:.3f} ms", flush=True)
