"""Relative parity of the product BA kernels against the oracle at the scales
the bench and DPVO run: per case the last iteration's
pose step dX (fp64 tangent) and the total pose / inverse-depth deltas,
||got - ref|| / ||ref||.  One JSON line per case.

    python scripts/ba_parity_probe.py [--cfg4]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from dpvo_amd import fastba, synthetic  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    n = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / n) if n > 0 else float(np.linalg.norm(a - b))


def case(name, G, t0, t1, iters, mode, dev):
    D = G.to(dev)
    cb = fastba.cuda_ba
    lm = torch.tensor([1e-4], device=dev)
    poses, patches = D.poses.clone(), D.patches.clone()
    if mode == "forward":
        dx = cb.forward_dx(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk,
                           G.M, t0, t1, iters, False)
    else:  # the bench's call: fused reproject + order + plan, then BA(plan=ws)
        mem = int(D.jj.max().item()) + 1
        _, _, ws = fastba.reproject(poses, patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem,
                                    plan_window=(t0, t1))
        fastba.BA(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, t0, t1,
                  M=G.M, iterations=iters, plan=ws)
        dx = cb.last_dx(ws, int(D.ii.numel()), t0, t1)
    st = cb.check_status(poses)
    P, K, dX = poses.cpu().numpy(), patches.cpu().numpy(), dx.cpu().numpy()
    Pr, Kr, d = oracle.ba(G.poses.numpy(), G.patches.numpy(), G.intrinsics.numpy(),
                          G.target.numpy(), G.weight.numpy(), 1e-4, G.ii.numpy(), G.jj.numpy(),
                          G.kk.numpy(), t0, t1, iters, diagnostics=True)
    P0, K0 = G.poses.numpy(), G.patches.numpy()
    out = {"case": name, "E": int(G.E), "N": t1 - t0, "iters": iters, "mode": mode, "status": st,
           "dX_rel": rel(dX, d["dX"]), "dX_norm": float(np.linalg.norm(d["dX"])),
           "dP_rel": rel(P[t0:t1] - P0[t0:t1], Pr[t0:t1] - P0[t0:t1]),
           "dP_norm": float(np.linalg.norm(Pr[t0:t1] - P0[t0:t1])),
           "dP_maxabs": float(np.abs(P - Pr).max()),
           "dZ_rel": rel(K[:, 2] - K0[:, 2], Kr[:, 2] - K0[:, 2]),
           # ulp floor of the pose delta: one fp32 ulp of every free pose entry
           "dP_ulp_floor": float(np.linalg.norm(np.spacing(np.abs(Pr[t0:t1]).astype(np.float32)))
                                 / max(np.linalg.norm(Pr[t0:t1] - P0[t0:t1]), 1e-30))}
    print(json.dumps(out), flush=True)


def main():
    dev = torch.device("cuda:0")
    for it in (1, 2):
        G = synthetic.make_config("cfg2", seed=0)
        case("cfg2", G, 1, G.F, it, "bench", dev)
        case("cfg2", G, 1, G.F, it, "forward", dev)
        for M in (10, 18, 25):
            G = synthetic.make_dpvo_window(M=M, seed=M)
            case(f"dpvo{M}", G, G.F - 10, G.F, it, "forward", dev)
            case(f"dpvo{M}", G, G.F - 10, G.F, it, "bench", dev)
        G = synthetic.make_config("cfg4s", seed=0)
        case("cfg4s", G, 1, G.F, it, "forward", dev)
    if "--cfg4" in sys.argv:
        G = synthetic.make_config("cfg4", seed=0)
        case("cfg4", G, 1, G.F, 1, "forward", dev)


if __name__ == "__main__":
    main()
