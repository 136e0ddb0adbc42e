"""Timing of the training-path dense solve (spd_solve.hip through
cuda_ba.spd_solve: batched Cholesky + both sweeps, one workgroup per batch
item) against torch.linalg.cholesky_ex + cholesky_solve (rocSOLVER) on the
same SPD systems, HIP-event medians.  Shapes: ba.py's pose systems (6N x 6N,
N = 8 / 16, batch 1 and 8) and larger n with the HBM working copy.

    python scripts/spd_solve_bench.py [--reps 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dpvo_amd  # noqa: E402


def timed(fn, reps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    cb = dpvo_amd.load_extension("cuda_ba")
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    for B, n, k, dt in [(1, 48, 1, torch.float64), (8, 48, 1, torch.float64), (1, 96, 1, torch.float64),
                        (8, 96, 1, torch.float64), (1, 96, 1, torch.float32), (1, 200, 1, torch.float32),
                        (1, 300, 1, torch.float64)]:
        A = torch.randn(B, n, n, generator=g, dtype=torch.float64)
        H = (A @ A.transpose(-1, -2) + n * torch.eye(n, dtype=torch.float64)).to(dev, dt)
        b = torch.randn(B, n, k, generator=g, dtype=torch.float64).to(dev, dt)
        ours = timed(lambda: cb.spd_solve(H, b), args.reps)
        ref = timed(lambda: torch.cholesky_solve(b, torch.linalg.cholesky_ex(H)[0]), args.reps)
        x = cb.spd_solve(H, b)[0]
        xr = torch.cholesky_solve(b, torch.linalg.cholesky_ex(H)[0])
        rel = float((x - xr).norm() / xr.norm())
        print(json.dumps({"batch": B, "n": n, "rhs": k, "dtype": str(dt).split(".")[-1],
                          "spd_solve_us": round(ours, 1), "torch_rocsolver_us": round(ref, 1),
                          "rel_diff": rel}), flush=True)


if __name__ == "__main__":
    main()
