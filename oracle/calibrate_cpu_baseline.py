"""TEST / BASELINE INFRASTRUCTURE ONLY -- calibrate the cpu_baseline port
(oracle/cpu_baseline.py) against the reference's own CPU fallback code, run
here in the build container (the reference never travels to the GPU box).

Times, on the SURVEY 8(d) cfg2 inputs (2048 edges, 128 channels, 36-frame
feature ring, 120x160, levels [1, 4], R = 3, fp32), at torch.set_num_threads
2 (what DPVO.__init__ sets, dpvo/dpvo.py:66) and all cores:
  * the reference's corr_torch_forward (dpvo/altcorr/correlation_kernel.py:
    461-548, loaded by file path) for both levels, vs the port's
    corr_grid_sample on the same tensors (outputs compared too);
  * the port's BA (2 iterations).  The reference's ba.py needs lietorch /
    torch_scatter builds that are absent here, so its BA time is the survey's
    stand-in figure, quoted, not re-measured.
Writes profiles/r02_cpu_calibration.json.

    python oracle/calibrate_cpu_baseline.py
"""
import importlib.util
import json
import os
import sys
import time

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
import cpu_baseline  # noqa: E402
from dpvo_amd import synthetic  # noqa: E402

REF = "/root/reference/dpvo/altcorr/correlation_kernel.py"


def load_ref():
    spec = importlib.util.spec_from_file_location("ref_correlation_kernel", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def timed(fn, reps=1):
    fn()  # warm
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    return (time.perf_counter() - t) / reps, out


def main():
    ref = load_ref()
    G = synthetic.make_config("cfg2", seed=0)
    g = torch.Generator().manual_seed(0)
    mem, C, levels = 36, 128, (1, 4)
    f1 = 0.25 * torch.randn(1, mem, C, 120, 160, generator=g)
    pyr = [f1 if s == 1 else F.avg_pool2d(f1[0], s, s).unsqueeze(0) for s in levels]
    gmap = 0.25 * torch.randn(1, G.F * G.M, C, 3, 3, generator=g)
    coords = torch.stack([G.patches[G.kk, 0], G.patches[G.kk, 1]], 1).unsqueeze(0) + 0.37
    kk, jj = G.kk, G.jj % mem
    res = {"cpu_count": os.cpu_count(), "config": "cfg2: 2048 edges, C=128, mem=36, levels [1,4]",
           "runs": []}
    for thr in (2, os.cpu_count()):
        torch.set_num_threads(thr)
        t_ref, o_ref = timed(lambda: [ref.corr_torch_forward(gmap, p, coords / s, kk, jj, 3)
                                      for p, s in zip(pyr, levels)])
        t_port, o_port = timed(lambda: [cpu_baseline.corr_grid_sample(gmap, p, coords / s, kk, jj, 3)
                                        for p, s in zip(pyr, levels)])
        err = max(float((a - b).abs().max()) for a, b in zip(o_ref, o_port))
        t_ba, _ = timed(lambda: [cpu_baseline.ba_step(G.poses, G.patches, G.intrinsics[0],
                                                      G.target, G.weight, 1e-4, G.ii, G.jj, G.kk,
                                                      1) for _ in range(2)], reps=3)
        run = {"threads": thr, "ref_corr_s": t_ref, "port_corr_s": t_port,
               "port_over_ref_corr": t_port / t_ref, "corr_max_abs_diff": err,
               "port_ba_2it_s": t_ba}
        print(run, flush=True)
        res["runs"].append(run)
    res["survey_ref_ba_2it_s"] = {"8 threads": 0.0245, "2 threads": 0.0247,
                                  "note": "BASELINE.md 2 (survey stand-ins for lietorch / "
                                          "torch_scatter); not re-measurable here"}
    out = os.path.join(REPO, "profiles", "r02_cpu_calibration.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
