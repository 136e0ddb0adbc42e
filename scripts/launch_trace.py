"""Per-workgroup timeline of the fused frame insertion + reprojection + edge
order + BA plan launch (ba_window.hip reproject_plan_insert_kernel) inside the
bench's step (fused launch -> A-CORR -> BA window, cfg2 shapes).

Every workgroup stamps its start / end (100 MHz wall clock) when marks are on
(cuda_ba.set_marks); shard 0 of the plan also stamps its phases.  Prints, per
role, the median over steps of its first start, its last end and its longest
workgroup, relative to the launch's first start.

    python scripts/launch_trace.py [--steps 40]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dpvo_amd import altcorr, fastba, synthetic  # noqa: E402

def ba_phases(m, iters=2):
    """Workgroup 0's phase table of the BA window kernel (as ba_window_phases.py)."""
    d = {"BA kernel (marks)": m[63] - m[0], "setup": m[1] - m[0],
         "  plan entries + counts": m[40] - m[0], "  scan": m[41] - m[40],
         "  records": m[42] - m[41], "  patch values, edge ids, poses": m[43] - m[42],
         "  per-edge inputs": m[1] - m[43]}
    prev = 1
    for it in range(iters):
        mb = 2 + 8 * it
        d[f"it{it}: (apply+) assemble"] = m[mb + 4] - m[prev]
        d[f"it{it}: reduce + publish"] = m[mb] - m[mb + 4]
        d[f"it{it}: wait partials"] = m[mb + 1] - m[mb]
        d[f"it{it}: gather"] = m[mb + 2] - m[mb + 1]
        d[f"it{it}:   last granules"] = m[mb + 5] - m[mb + 1]
        d[f"it{it}:   sum shares"] = m[mb + 2] - m[mb + 5]
        d[f"it{it}: solve"] = m[mb + 3] - m[mb + 2]
        prev = mb + 3
    d["final apply + write-back"] = m[63] - m[prev]
    return {k: v * 0.01 for k, v in d.items()}


PHASES = ["edge pass", "histogram", "local scan", "scatter", "block work", "rank + stores"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--separate-insert", action="store_true",
                    help="insert the frame in its own launch (the reprojection + plan launch "
                         "has no workgroup marks then: plan phases only)")
    args = ap.parse_args()
    cb = fastba.cuda_ba
    dev = torch.device("cuda:0")
    mem, levels = 36, [1, 2, 4, 8]
    G = synthetic.make_config(args.config, seed=0)
    D = G.to(dev)
    P = G.patches.shape[-1]
    pyr_nchw = synthetic.make_features(mem=mem, C=128, levels=levels, seed=0, device=dev)
    pyr = [synthetic.channels_last(p) for p in pyr_nchw]
    gbuf = torch.randn(1, mem * G.M, 128, P, P, device=dev)
    lmbda = torch.tensor([1e-4], device=dev)
    poses, patches = D.poses.clone(), D.patches.clone()
    kk1, jj1 = D.kk % (G.M * mem), D.jj % mem
    scales = [float(s) for s in levels]
    E = int(D.ii.numel())
    nps = 1 if E <= 512 else min((E + 511) // 512, 16)
    nrep = (E * P * P + 511) // 512

    def step(i):
        if args.separate_insert:
            altcorr.insert_frame(pyr_nchw[0][0, i % mem], pyr, i % mem, levels)
            coords, order, ws = fastba.reproject(poses, patches, D.intrinsics, D.ii, D.jj, D.kk,
                                                 mem=mem, plan_window=(1, G.F))
        else:
            coords, order, ws = fastba.reproject(
                poses, patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem, plan_window=(1, G.F),
                insert=(pyr_nchw[0][0, i % mem], [p[0, i % mem] for p in pyr], levels))
        altcorr.corr_levels(gbuf, pyr, coords, kk1, jj1, 3, scales, order=order)
        fastba.BA(poses, patches, D.intrinsics, D.target, D.weight, lmbda, D.ii, D.jj, D.kk, 1,
                  G.F, M=G.M, iterations=2, plan=ws)
        return ws

    for i in range(20):
        step(i)
    torch.cuda.synchronize()
    off = cb.plan_offsets(E, 1, G.F)
    rows, phases, ba = [], [], []
    cb.set_marks(True)
    try:
        for i in range(args.steps):
            ws = step(i)
            torch.cuda.synchronize()
            allm = cb.workspace_marks(ws, E, 1, G.F).cpu().numpy()
            ba.append(ba_phases(allm.tolist()))
            mk = allm[1664:].reshape(-1, 2)
            b = ws.cpu().numpy().tobytes()
            st = np.frombuffer(b[off[4] + 64:off[4] + 64 + 72], np.int64)
            ph = np.diff(st[:7]) * 0.01
            phases.append(np.append(ph, (st[8] - st[7]) / max(ph.sum(), 1e-3)))
            rows.append(mk.copy())
    finally:
        cb.set_marks(False)
    m = np.median(np.array(phases), axis=0)
    plan_line = ("  plan shard 0 phases: " + ", ".join(f"{n} {x:.2f}" for n, x in zip(PHASES, m))
                 + f" us; total {m[:-1].sum():.2f} us; shader clock {m[-1]:.0f} MHz")
    ba_lines = [f"  {k:34s} median {np.median([d[k] for d in ba]):6.2f} us" for k in ba[0]]
    if args.separate_insert:
        print(f"{args.config}: E={E}, frame insertion in its own launch")
        print(plan_line)
        print("BA window kernel in the step (workgroup 0):")
        print("\n".join(ba_lines))
        return
    # workgroups >= 256 carry no marks (the launch stamps blockIdx < 256 only;
    # the rows past 256 hold other marks): the timeline covers the first 256
    nwg = min(256, int(max((r[:256, 0] > 0).sum() for r in rows)))
    roles = {"plan shards": range(0, nps), "edge order": range(nps, nps + 1),
             "reprojection": range(nps + 1, nps + 1 + nrep),
             "insertion": range(nps + 1 + nrep, nwg)}
    print(f"{args.config}: E={E} marked workgroups={nwg} (plan {nps}, order 1, reprojection "
          f"{nrep}, insertion {nwg - nps - 1 - nrep} of the launch's first 256)")
    stats = {k: [] for k in roles}
    span = []
    for r in rows:
        r = r[:nwg].astype(np.int64)
        t0 = r[:, 0].min()
        span.append((r[:, 1].max() - t0) * 0.01)
        for k, idx in roles.items():
            idx = list(idx)
            if not idx:
                continue
            s, e = r[idx, 0] - t0, r[idx, 1] - t0
            stats[k].append((s.min() * 0.01, e.max() * 0.01, (e - s).max() * 0.01,
                             np.median(s) * 0.01))
    print(f"launch span (first start -> last end) median {np.median(span):.2f} us")
    for k, v in stats.items():
        if not v:
            continue
        m = np.median(np.array(v), axis=0)
        print(f"  {k:14s} first start {m[0]:5.2f}  median start {m[3]:5.2f}  last end {m[1]:5.2f}"
              f"  longest workgroup {m[2]:5.2f} us")
    print(plan_line)
    print("BA window kernel in the step (workgroup 0):")
    print("\n".join(ba_lines))


if __name__ == "__main__":
    main()
