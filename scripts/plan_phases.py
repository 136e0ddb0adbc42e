"""Phase stamps of the sharded BA plan (shard 0, 100 MHz wall clock): edge
pass (loads + kmin/kmax/fmin), presence bitmap + local histogram, local scan,
scatter, rank + stores -- alone (fastba.plan) and inside the fused
insert + reproject + order + plan launch.

    python scripts/plan_phases.py [cfg2|dpvo25 ...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dpvo_amd import fastba, synthetic  # noqa: E402
from dpvo_amd._native import load_extension  # noqa: E402

NAMES = ["edge pass", "presence + histogram", "local scan", "scatter", "block work", "rank + stores"]


def stamps(cb, ws, E, t0, t1):
    off = cb.plan_offsets(E, t0, t1)
    b = ws.cpu().numpy().tobytes()
    return np.frombuffer(b[off[4] + 64:off[4] + 64 + 72], np.int64)


def main():
    cb = load_extension("cuda_ba")
    dev = torch.device("cuda:0")
    mem, levels = 36, (1, 2, 4, 8)
    pyr_nchw = synthetic.make_features(mem=mem, C=128, levels=levels, seed=0, device=dev)
    pyr = [synthetic.channels_last(p) for p in pyr_nchw]
    for name in (sys.argv[1:] or ["cfg2", "dpvo25"]):
        if name == "cfg2":
            G = synthetic.make_config("cfg2", seed=0)
            t0, t1 = 1, G.F
        else:
            G = synthetic.make_dpvo_window(M=25, seed=25)
            t0, t1 = G.F - 10, G.F
        D = G.to(dev)
        ins = (pyr_nchw[0][0, 3], [p[0, 3] for p in pyr], levels)
        runs = {
            "plan alone": lambda: fastba.plan(D.ii, D.jj, D.kk, t0, t1, D.patches.shape[0],
                                              D.poses.shape[0]),
            "fused launch": lambda: fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj,
                                                     D.kk, mem=mem, plan_window=(t0, t1),
                                                     insert=ins)[2],
        }
        for k, fn in runs.items():
            rows = []
            for rep in range(40):
                ws = fn()
                torch.cuda.synchronize()
                if rep >= 10:
                    st = stamps(cb, ws, G.E, t0, t1)
                    ph = np.diff(st[:7]) * 0.01
                    # shader-clock cycles / wall us over the plan = clock in MHz
                    rows.append(np.append(ph, (st[8] - st[7]) / max(ph.sum(), 1e-3)))
            med = np.median(np.array(rows), axis=0)
            print(f"{name} E={G.E} {k}: " + ", ".join(f"{n} {v:.2f}" for n, v in zip(NAMES, med))
                  + f" us; total {med[:-1].sum():.2f} us; shader clock {med[-1]:.0f} MHz",
                  flush=True)


if __name__ == "__main__":
    main()
