"""Per-phase timing of the default F-BA path (ba_blocks.hip) on cfg2: CUDA-event
total per call plus the wall-clock stamps workgroup 0 leaves (100 MHz clock):

  0 start, 40 loads, 41 sort, 42 carve, 1 setup end,
  per iteration it (mb = 2 + 8 it): mb+0 assembled, mb+1 block stored,
  mb+2 all blocks arrived, mb+3 gathered, mb+4 factored, mb+5 solved,
  mb+6 dX published; 63 end.

    python scripts/ba_blocks_phases.py [cfg] [iterations] [solve mode]
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
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # dense solve: 0 fp32, 1 fp32+refine, 2 fp64 LDL
cb.set_refine(mode)
print(f"solve mode {mode}")
G = synthetic.make_config(cfg, seed=0)
D = G.to(dev)
lm = torch.tensor([1e-4], device=dev)
acc = {}
for rep in range(40):
    poses, patches = D.poses.clone(), D.patches.clone()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    cb.forward(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk, G.M, 1,
               G.F, iters, False)
    e1.record()
    torch.cuda.synchronize()
    poses, patches = D.poses.clone(), D.patches.clone()
    m = cb.forward_marks(poses, patches, D.intrinsics, D.target, D.weight, lm, D.ii, D.jj, D.kk,
                         G.M, 1, G.F, iters, False).cpu().tolist()
    if rep < 5:
        continue
    d = {"call (events)": e0.elapsed_time(e1) * 1e3}
    seq = [("setup: loads", 0, 40), ("setup: sort", 40, 41), ("setup: scan/carve", 41, 42),
           ("setup: records", 42, 1)]
    prev = 1
    for it in range(iters):
        mb = 2 + 8 * it
        if it > 0:
            seq.append((f"it{it}: apply prev", prev, mb - 8 + 6 + 0) if False else
                       (f"it{it}: publish->assembled", prev, mb))
        else:
            seq.append((f"it{it}: assemble", prev, mb))
        seq += [(f"it{it}: reduce+store", mb, mb + 1), (f"it{it}: wait arrivals", mb + 1, mb + 2),
                (f"it{it}: gather", mb + 2, mb + 3), (f"it{it}: factor", mb + 3, mb + 4),
                (f"it{it}: backsub", mb + 4, mb + 5), (f"it{it}: publish", mb + 5, mb + 6)]
        prev = mb + 6
    seq.append(("final apply + writeback", prev, 63))
    seq.append(("kernel total (marks)", 0, 63))
    for name, a, b in seq:
        d[name] = (m[b] - m[a]) * 0.01
    for k, v in d.items():
        acc.setdefault(k, []).append(v)
for k, v in acc.items():
    v = sorted(v)
    print(f"{k:32s} median {v[len(v) // 2]:8.2f} us")
