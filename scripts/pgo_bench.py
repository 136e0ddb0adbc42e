"""Timing of cuda_ba.solve_system (Sim3 pose graph, ba.cpp:120-180) on the
device, median of HIP-event timings of the whole call (host plan, block
assembly, segment sweeps, border Cholesky).  Graphs (tests/test_pgo.py
generators): "loop graph" = odometry chain + n/50 long loop edges (the shape
loop closure builds); "random 3n edges" = chain + 2n random edges (nearly every
pose on the border: the dense worst case)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dpvo_amd  # noqa: E402
from test_pgo import make_loop_graph, make_pgo  # noqa: E402

cb = dpvo_amd.load_extension("cuda_ba")
dev = torch.device("cuda:0")
cases = [("loop graph", n, make_loop_graph(n, n // 50, seed=0)) for n in (100, 500, 1000, 2000, 4000)]
cases += [("random 3n edges", n, make_pgo(n, 3 * n, seed=0)) for n in (100, 500, 1000, 2000)]
for kind, n, g in cases:
    r = len(g[2])
    Ji, Jj, ii, jj, res = [torch.from_numpy(a).to(dev) for a in g]
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
    print(f"solve_system {kind:16s} n={n} r={r}: {sorted(ts)[5]:.3f} ms", flush=True)
