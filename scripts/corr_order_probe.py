"""A-CORR edge-order probe (cfg2, channels-last fp32/fp16): HIP-event median of
the per-level kernel for different edge orders handed to corr_levels --
the device order (edges grouped by target frame), and orders that also sort
the edges of a frame by where their patch lands (row-major cells of a given
size, Morton), or shuffle them.  Every order gives the same outputs (each
edge is computed on its own); only L2 reuse between concurrent waves changes.

    python scripts/corr_order_probe.py [--reps 200] [--features f32]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from dpvo_amd import altcorr, fastba, synthetic  # noqa: E402


def morton(x, y):
    def spread(v):
        v = v & 0xFF
        v = (v | (v << 4)) & 0x0F0F
        v = (v | (v << 2)) & 0x3333
        v = (v | (v << 1)) & 0x5555
        return v
    return spread(x) | (spread(y) << 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--features", default="f32")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    G = synthetic.make_config("cfg2", seed=0)
    D = G.to(dev)
    mem, P, C = 36, 3, 128
    levels = [1, 2, 4, 8]
    coords, order_dev = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem)
    kk1, jj1 = D.kk % (G.M * mem), D.jj % mem
    E = G.E
    cx = coords[0, :, 0, P // 2, P // 2].clamp(0, 159).long()
    cy = coords[0, :, 1, P // 2, P // 2].clamp(0, 119).long()
    f = jj1.long()
    orders = {"device": order_dev}
    for cs in (8, 16, 32, 64):
        key = (f * 1000 + (cy // cs) * 100 + (cx // cs)) * 4096 + torch.arange(E, device=dev)
        orders[f"rows{cs}"] = torch.argsort(key).int()
    mk = torch.tensor([morton(int(x) // 4, int(y) // 4) for x, y in zip(cx.tolist(), cy.tolist())],
                      device=dev)
    orders["morton4"] = torch.argsort(f * (1 << 20) + mk * 4096 + torch.arange(E, device=dev)).int()
    g = torch.Generator(device="cpu").manual_seed(0)
    rnd = torch.randperm(E, generator=g).to(dev)
    orders["frame_shuffled"] = torch.argsort(f * 4096 + rnd).int()
    orders["unsorted"] = torch.arange(E, device=dev, dtype=torch.int32)
    for feat in args.features.split(","):
        fdt = torch.float16 if feat == "f16" else torch.float32
        pyr = [synthetic.channels_last(p) for p in
               synthetic.make_features(mem=mem, C=C, levels=levels, seed=0, device=dev, dtype=fdt)]
        gbuf = (0.25 * torch.randn(1, mem * G.M, C, P, P, device=dev)).to(fdt)
        ref = None
        for rnd_ in range(2):
            for name, od in orders.items():
                run = lambda: altcorr.corr_levels(gbuf, pyr, coords, kk1, jj1, 3,  # noqa: E731
                                                  [float(s) for s in levels], order=od)
                for _ in range(20):
                    run()
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(args.reps)]
                for a, b in ev:
                    a.record()
                    run()
                    b.record()
                torch.cuda.synchronize()
                ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
                out = run()
                if ref is None:
                    ref = out.clone()
                same = bool(torch.equal(out, ref))
                print(json.dumps({"features": feat, "order": name, "round": rnd_,
                                  "us_median": round(ts[len(ts) // 2], 2),
                                  "us_min": round(ts[0], 2), "bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()
