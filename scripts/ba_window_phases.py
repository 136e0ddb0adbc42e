"""Per-phase timing of the default F-BA path (ba_window.hip) from the
wall-clock stamps (100 MHz) workgroup 0 leaves: [0] start, [1] setup done,
per iteration (mb = 2 + 8 it): mb+0 block assembled + reduced + stored,
mb+1 every partial arrived, mb+2 S gathered, mb+3 solved; [63] end.
The plan kernel runs before [0] (its time is in 'call - kernel').

    python scripts/ba_window_phases.py [cfg|M] [iterations]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import dpvo_amd  # noqa: E402
from dpvo_amd import synthetic  # noqa: E402

cb = dpvo_amd.load_extension("cuda_ba")
dev = torch.device("cuda:0")
arg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
if arg.startswith("cfg"):
    G = synthetic.make_config(arg, seed=0)
    t0, t1 = 1, G.F
else:
    G = synthetic.make_dpvo_window(M=int(arg), seed=int(arg))
    t0, t1 = G.F - 10, G.F
D = G.to(dev)
lm = torch.tensor([1e-4], device=dev)
acc = {}
for rep in range(40):
    poses, patches = D.poses.clone(), D.patches.clone()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cb.forward(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, G.M, t0, t1,
               iters, False)
    e1.record()
    torch.cuda.synchronize()
    poses, patches = D.poses.clone(), D.patches.clone()
    m = cb.forward_marks(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk,
                         G.M, t0, t1, iters, False).cpu().tolist()
    if rep < 5:
        continue
    d = {"call (events)": e0.elapsed_time(e1) * 1e3, "kernel (marks)": (m[63] - m[0]) * 0.01,
         "setup": (m[1] - m[0]) * 0.01,
         "  setup: plan entries + counts": (m[40] - m[0]) * 0.01,
         "  setup: scan": (m[41] - m[40]) * 0.01,
         "  setup: records": (m[42] - m[41]) * 0.01,
         "  setup: patch values, edge ids, poses": (m[43] - m[42]) * 0.01,
         "  setup: per-edge inputs": (m[1] - m[43]) * 0.01}
    prev = 1
    for it in range(iters):
        mb = 2 + 8 * it
        d[f"it{it}: (apply+) assemble"] = (m[mb + 4] - m[prev]) * 0.01
        d[f"it{it}: reduce + publish"] = (m[mb] - m[mb + 4]) * 0.01
        d[f"it{it}: wait partials"] = (m[mb + 1] - m[mb]) * 0.01
        d[f"it{it}: gather"] = (m[mb + 2] - m[mb + 1]) * 0.01
        d[f"it{it}:   last granules"] = (m[mb + 5] - m[mb + 1]) * 0.01
        d[f"it{it}:   sum shares"] = (m[mb + 2] - m[mb + 5]) * 0.01
        d[f"it{it}: solve"] = (m[mb + 3] - m[mb + 2]) * 0.01
        prev = mb + 3
    d["final apply + write-back"] = (m[63] - m[prev]) * 0.01
    for k, v in d.items():
        acc.setdefault(k, []).append(v)
print(f"{arg}: E={G.E} N={t1 - t0} iterations={iters}")
for k, v in acc.items():
    v = sorted(v)
    print(f"{k:34s} median {v[len(v) // 2]:8.2f} us")

# final apply of workgroup 0: poses retracted, E entries staged, depths updated, end
if m[48] and m[50] and m[63] > m[50]:
    mf = 2 + 8 * (iters - 1) + 3
    print(f"final apply wg0: poses {(m[48] - m[mf]) * 0.01:.2f} us, depths "
          f"{(m[50] - m[49]) * 0.01:.2f} us, write-back + status {(m[63] - m[50]) * 0.01:.2f} us"
          f" (relevant edges {m[52]}, E entries {'in HBM' if m[53] & 1 else 'in LDS'})")

# per-workgroup spread (window kernel stamps [128 + 256 it + g] assembled,
# [640 + 256 it + g] every partial seen), last call
if m[128] and len(m) >= 1664:
    import statistics

    G = sum(1 for g in range(256) if m[128 + g])
    for it in range(min(iters, 2)):
        asm = [(m[128 + 256 * it + g] - m[0]) * 0.01 for g in range(G)]
        seen = [(m[640 + 256 * it + g] - m[0]) * 0.01 for g in range(G)]
        order = sorted(range(G), key=lambda g: asm[g])
        print(f"it{it}: {G} workgroups assembled at {min(asm):.2f}..{max(asm):.2f} us "
              f"(median {statistics.median(asm):.2f}); all partials seen at "
              f"{min(seen):.2f}..{max(seen):.2f} us; slowest workgroups {order[-5:]}")
    setup = [(m[1152 + g] - m[0]) * 0.01 for g in range(G)]
    pre = [(m[1408 + g] - m[0]) * 0.01 for g in range(G)]
    print(f"setup done at {min(setup):.2f}..{max(setup):.2f} us (median "
          f"{statistics.median(setup):.2f}); it0 pre-reduction at {min(pre):.2f}..{max(pre):.2f} "
          f"(median {statistics.median(pre):.2f})")
    if len(m) >= 2432 and m[2176]:
        ends = [(m[2176 + g] - m[0]) * 0.01 for g in range(G)]
        print(f"workgroup ends at {min(ends):.2f}..{max(ends):.2f} us (median "
              f"{statistics.median(ends):.2f}; workgroup 0 at {(m[63] - m[0]) * 0.01:.2f}); "
              f"last workgroups {sorted(range(G), key=lambda g: ends[g])[-5:]}")
    print("per workgroup (g: setup, pre-reduce, assembled, seen):",
          [(g, round(setup[g], 2), round(pre[g], 2), round((m[128 + g] - m[0]) * 0.01, 2),
            round((m[640 + g] - m[0]) * 0.01, 2)) for g in order[-8:]])
