"""CPU: the bench's cpu_baseline leg (oracle/cpu_baseline.py, a torch-CPU
restatement of the reference's fallback op sequence) pinned to the
reference's own outputs, so the reported CPU number measures the reference's
computation:
  * corr_grid_sample vs corr_torch_forward (correlation_kernel.py:461-548),
    fixture corr_gs_a;
  * ba_step vs dpvo/ba.py BA (88-297) run by oracle/make_golden.py with ep=1.0
    and the +-64 px bounds, in fp64 (tight) and fp32 (loose: the
    reference's own fp32 noise)."""
import numpy as np
import pytest
import torch
from conftest import golden

import cpu_baseline


def test_corr_port_matches_reference_grid_sample():
    z = golden("corr_gs_a")
    out = cpu_baseline.corr_grid_sample(torch.from_numpy(z["fmap1"]), torch.from_numpy(z["fmap2"]),
                                        torch.from_numpy(z["coords"]), torch.from_numpy(z["ii"]),
                                        torch.from_numpy(z["jj"]), int(z["radius"]))
    np.testing.assert_allclose(out.numpy(), z["out"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("name", ["ba_py_a", "ba_py_b"])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_ba_port_matches_reference_ba_py(name, dtype):
    z = golden(name)
    t = lambda k: torch.from_numpy(np.asarray(z[k])).to(dtype)  # noqa: E731
    cx, cy = float(z["intrinsics"][0, 2]), float(z["intrinsics"][0, 3])
    P, K = cpu_baseline.ba_step(t("poses"), t("patches"), t("intrinsics")[0], t("target"),
                                t("weight"), 1e-4, torch.from_numpy(z["ii"]),
                                torch.from_numpy(z["jj"]), torch.from_numpy(z["kk"]), int(z["t0"]),
                                ep=1.0, bounds=(-64.0, -64.0, 2 * cx + 64.0, 2 * cy + 64.0))
    if dtype == torch.float64:
        np.testing.assert_allclose(P.numpy(), z["out_poses64"], rtol=0, atol=1e-7)
        np.testing.assert_allclose(K.numpy(), z["out_patches64"], rtol=1e-5, atol=1e-7)
    else:
        np.testing.assert_allclose(P.numpy(), z["out_poses"], rtol=0, atol=5e-5)
        # fp32 vs the reference's fp32 run: both carry fp32 Schur-solve noise
        # (condition ~1e5): 99% of depths within 5e-3, none beyond 2e-2
        d = np.abs(K.numpy() - z["out_patches"])
        assert np.quantile(d, 0.99) < 5e-3 and d.max() < 2e-2, (np.quantile(d, 0.99), d.max())
