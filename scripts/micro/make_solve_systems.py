"""Dump damped Schur systems (S in lower 6x6-block layout, y) of the oracle
for the window-solver micro-benchmarks (gj_bench.hip): cfg2 seeds 0 / 4 and
DPVO windows M = 10 / 25.  Test infrastructure (imports the oracle)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from dpvo_amd import synthetic  # noqa: E402


def dump(name, G, t0, t1):
    P, K, d = oracle.ba(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(), G.target.numpy(),
                        G.weight.numpy(), 1e-4, G.ii.numpy(), G.jj.numpy(), G.kk.numpy(), t0, t1, 1,
                        diagnostics=True)
    S, y, N = d["S"], d["y"], t1 - t0
    blocks = []
    for a in range(N):
        for b in range(a + 1):
            blocks.append(S[6 * a:6 * a + 6, 6 * b:6 * b + 6].reshape(-1))
    with open(os.path.join(HERE, "data", name + ".bin"), "wb") as f:
        np.array([N], np.int32).tofile(f)
        np.concatenate(blocks).astype(np.float64).tofile(f)
        y.astype(np.float64).tofile(f)
        np.linalg.solve(S, y).astype(np.float64).tofile(f)
    print(name, N, "cond %.3g" % np.linalg.cond(S))


def main():
    for s in (0, 4):
        G = synthetic.make_config("cfg2", seed=s)
        dump(f"cfg2_s{s}", G, 1, G.F)
    for M in (10, 25):
        G = synthetic.make_dpvo_window(M=M, seed=M)
        dump(f"dpvo{M}", G, G.F - 10, G.F)


if __name__ == "__main__":
    main()
