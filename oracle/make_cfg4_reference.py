"""TEST INFRASTRUCTURE ONLY -- oracle result for the full BASELINE cfg4 graph
(1024 frames x 96 patches, ~131k edges, N = 1023 free poses), one BA
iteration, for tests/test_ba_large_gpu.py::test_cfg4_full_size_matches_oracle.

The oracle (oracle/dpvo_oracle.c, ba_cuda.cu semantics with a dense fp64 S and
Cholesky) takes minutes at this size, so it runs here once and the committed
fixture holds only its outputs (poses, inverse depths, the pose step dX)
plus a digest of the inputs; the test rebuilds
the inputs from the same seed (dpvo_amd.synthetic, torch CPU generator) and
checks the digest before comparing.

    python oracle/make_cfg4_reference.py
"""
import hashlib
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from dpvo_amd import synthetic  # noqa: E402


def digest(G):
    h = hashlib.sha256()
    for a in (G.poses, G.patches, G.intrinsics, G.ii, G.jj, G.kk, G.target, G.weight):
        h.update(np.ascontiguousarray(a.numpy()).tobytes())
    return h.hexdigest()


def main():
    G = synthetic.make_config("cfg4", seed=0)
    t0, t1 = 1, G.F
    t = time.time()
    P, K, d = oracle.ba(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(),
                        G.target.numpy(), G.weight.numpy(), 1e-4, G.ii.numpy(), G.jj.numpy(),
                        G.kk.numpy(), t0, t1, 1, diagnostics=True)
    dt = time.time() - t
    out = os.path.join(REPO, "tests", "golden", "cfg4_ba1.npz")
    np.savez_compressed(out, poses=P.astype(np.float32), depth=K[:, 2, 1, 1].astype(np.float32),
                        depth00=K[:, 2, 0, 0].astype(np.float32), dX=d["dX"].astype(np.float64),
                        digest=digest(G), t0=t0, t1=t1,
                        E=G.E, seconds=dt)
    print("cfg4 oracle, 1 iteration:", round(dt, 1), "s, E", G.E, "->", out)


if __name__ == "__main__":
    main()
