"""A-CORR kernel variants on the bench's exact cfg2 call (channels-last
pyramid, levels [1,2,4,8], 2048 edges, XCD order): HIP-event median per
launch and the max deviation of each variant from the fp64 oracle sample.

    python scripts/corr_variants.py [--reps 200] [--variants 0,1,2,3] [--features f32]

variant 0: one wave per edge (corr_nhwc_kernel, split-f16 products)
variant 1: one wave per (edge, level), exact fp32 products (v_mfma_f32_16x16x4_f32)
variant 2: one wave per (edge, level), split-f16 products
variant 3: variant 1 with a 3-deep tile ring
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from dpvo_amd import _native, altcorr, fastba, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--variants", default="0,1,3")
    ap.add_argument("--features", default="f32")
    ap.add_argument("--levels", default="1,2,4,8")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _native.c_abi()
    G = synthetic.make_config("cfg2", seed=0)
    D = G.to(dev)
    mem, P, C = 36, 3, 128
    levels = [int(x) for x in args.levels.split(",")]
    fdt = torch.float16 if args.features == "f16" else torch.float32
    pyr_nchw = synthetic.make_features(mem=mem, C=C, levels=levels, seed=0, device=dev, dtype=fdt)
    pyr = [synthetic.channels_last(p) for p in pyr_nchw]
    gbuf = (0.25 * torch.randn(1, mem * G.M, C, P, P, device=dev)).to(fdt)
    coords, order = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem)
    kk1, jj1 = D.kk % (G.M * mem), D.jj % mem
    sc = [float(s) for s in levels]
    run = lambda: altcorr.corr_levels(gbuf, pyr, coords, kk1, jj1, 3, sc, order=order)  # noqa: E731
    outs = {}
    for v in [int(x) for x in args.variants.split(",")]:
        lib.dpvo_corr_nhwc_variant(v)
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
        outs[v] = run().clone()
        dev0 = None
        if 0 in outs and v != 0:
            ref = outs[0]
            dev0 = ((outs[v] - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps({"variant": v, "features": args.features, "levels": levels,
                          "us_median": ts[len(ts) // 2], "us_min": ts[0],
                          "max_dev_vs_v0_rel": dev0}), flush=True)
    lib.dpvo_corr_nhwc_variant(1)


if __name__ == "__main__":
    main()
