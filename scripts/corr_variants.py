"""A-CORR product kernels on the bench's exact cfg2 call (channels-last
pyramid, levels [1,2,4,8], 2048 edges, XCD order): HIP-event median per
launch for fp32 features (corr_nhwc_lvl_kernel, exact fp32 products) and fp16
features (the same kernel, fp16 MFMA), and the max deviation from the fp64 oracle on a
sample of edges.

    python scripts/corr_variants.py [--reps 200] [--features f32,f16] [--native DIR]

--native DIR loads the extension modules from another build directory (a
copy of dpvo_amd/_native built from another tree) for A/B runs in one call.

(Round 6's A/B of the per-edge split-f16 kernel against the per-level kernel
is in profiles/r06_mid/corr_variants.txt.)
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dpvo_amd._native as _nat  # noqa: E402

if "--native" in sys.argv:
    _nat.NATIVE_DIR = os.path.abspath(sys.argv[sys.argv.index("--native") + 1])

from dpvo_amd import altcorr, fastba, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--features", default="f32,f16")
    ap.add_argument("--levels", default="1,2,4,8")
    ap.add_argument("--native", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    G = synthetic.make_config("cfg2", seed=0)
    D = G.to(dev)
    mem, P, C = 36, 3, 128
    levels = [int(x) for x in args.levels.split(",")]
    coords, order = fastba.reproject(D.poses, D.patches, D.intrinsics, D.ii, D.jj, D.kk, mem=mem)
    kk1, jj1 = D.kk % (G.M * mem), D.jj % mem
    sc = [float(s) for s in levels]
    for feat in args.features.split(","):
        fdt = torch.float16 if feat == "f16" else torch.float32
        pyr_nchw = synthetic.make_features(mem=mem, C=C, levels=levels, seed=0, device=dev, dtype=fdt)
        pyr = [synthetic.channels_last(p) for p in pyr_nchw]
        gbuf = (0.25 * torch.randn(1, mem * G.M, C, P, P, device=dev)).to(fdt)
        run = lambda: altcorr.corr_levels(gbuf, pyr, coords, kk1, jj1, 3, sc, order=order)  # noqa: E731
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
        out = run().view(1, G.E, 7, 7, P, P, len(levels)).double().cpu().numpy()
        dev_max = None
        try:
            import oracle

            sel = np.arange(0, G.E, 61)
            f1 = gbuf.float().cpu().numpy()
            worst = 0.0
            for l, s in enumerate(sc):
                ref = oracle.corr_fwd(f1, pyr_nchw[l].float().cpu().numpy(),
                                      (coords / s).cpu().numpy()[:, sel], kk1.cpu().numpy()[sel],
                                      jj1.cpu().numpy()[sel], 3)
                worst = max(worst, float(np.abs(out[..., l][:, sel] - ref).max() / np.abs(ref).max()))
            dev_max = worst
        except Exception as e:  # the oracle is a checker only; timing stands without it
            dev_max = f"oracle unavailable: {e}"
        print(json.dumps({"native": args.native or "in-tree", "features": feat, "levels": levels, "us_median": ts[len(ts) // 2],
                          "us_min": ts[0], "max_dev_vs_oracle_rel_sample": dev_max}), flush=True)


if __name__ == "__main__":
    main()
