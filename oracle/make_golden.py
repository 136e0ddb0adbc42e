"""TEST INFRASTRUCTURE ONLY -- generates the committed golden fixtures in
tests/golden/ by running the reference's OWN Python code from
/root/reference (read-only; no bytecode is written there).

Run in the build container (the reference does not exist on the GPU box):

    python oracle/make_golden.py

Fixtures (numpy .npz, inputs + expected outputs, seeded):
  corr_loop_*.npz      dpvo/altcorr/correlation_kernel.py corr_forward_torch_wrapper
                        (388-458): literal loop restatement of corr_forward_kernel
                        + host bilinear/permute (correlation_kernel.cu:82-175, 232-272)
  corr_gs_*.npz        correlation_kernel.py corr_torch_forward (461-548), fp32
                        grid_sample restatement, larger edge counts
  patchify_*.npz       correlation_kernel.py patchify_forward_kernel_CPU (141-178,
                        zero fill = CUDA semantics) and patchify_forward_kernel_python
                        (181-224, the fork's clamping runtime path)
  ba_py_*.npz          dpvo/ba.py BA (88-297), one LM step, run with ep=1.0 and
                        bounds = (-64,-64,2cx+64,2cy+64) on inputs where the
                        ba.py <-> ba_cuda.cu divergences are inert (SURVEY 8a A-BA-PY);
                        lietorch_backends is provided by the build's own CPU SE3
                        restatement (oracle/dpvo_oracle.c), torch_scatter by index_add_.
  transform_*.npz      dpvo/projective_ops.py transform (53-113) coords + Jacobians.
  keyframe_a.npz       dpvo/projective_ops.py flow_mag (120-130) on DPVO-window edges
                        (motionmag's input, dpvo.py:586-599) and at patch pixel (1, 1)
                        on the edges_loop candidates; the edges_loop composition
                        (patchgraph.py:74-91: flow_mag -> einops reduce -> mask ->
                        reduce_edges) and reduce_edges (loop_closure/optim_utils.py:
                        24-60) on a crafted case.  optim_utils is imported with numba
                        (absent) replaced by a pass-through njit and pypose (absent,
                        unused by reduce_edges) by an empty module.

    python oracle/make_golden.py [corr] [patchify] [ba] [keyframe]   (default: all)
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, HERE)
import oracle  # noqa: E402


def load_corr_module():
    path = os.path.join(REF, "dpvo", "altcorr", "correlation_kernel.py")
    spec = importlib.util.spec_from_file_location("ref_correlation_kernel", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# ----------------------------------------------------------------- stubs
def _make_lietorch_backends():
    """A CPU `lietorch_backends` backed by the C restatement (double)."""
    m = types.ModuleType("lietorch_backends")

    def fwd(op):
        def f(group_id, X, *rest):
            y = rest[0].detach().double().cpu().numpy() if rest else None
            out = oracle.lie_fwd(group_id, op, X.detach().double().cpu().numpy(), y)
            if op == "matrix":
                out = out.reshape(-1, 4, 4)
            return torch.from_numpy(out).to(X.dtype)
        return f

    def bwd(op):
        def f(group_id, grad, X, *rest):
            y = rest[0].detach().double().cpu().numpy() if rest else None
            outs = oracle.lie_bwd(group_id, op, grad.detach().double().cpu().numpy(),
                                  X.detach().double().cpu().numpy(), y)
            return [torch.from_numpy(o).to(X.dtype) for o in outs]
        return f

    for name, op in [("expm", "exp"), ("logm", "log"), ("inv", "inv"), ("mul", "mul"),
                     ("adj", "adj"), ("adjT", "adjT"), ("act", "act"), ("act4", "act4")]:
        setattr(m, name, fwd(op))
        setattr(m, name + "_backward", bwd(op))
    m.as_matrix = fwd("matrix")
    m.Jinv = fwd("Jinv")

    def projector(group_id, X):
        K, N = oracle.GROUP_DIMS[group_id]
        out = oracle.lie_fwd(group_id, "projector", X.detach().double().numpy())
        return torch.from_numpy(out.reshape(-1, N, N)).to(X.dtype)

    m.projector = projector
    return m


def _make_torch_scatter():
    m = types.ModuleType("torch_scatter")

    def scatter_sum(src, index, dim=-1, dim_size=None):
        dim = dim % src.dim()
        if dim_size is None:
            dim_size = int(index.max()) + 1 if index.numel() else 0
        shape = list(src.shape)
        shape[dim] = dim_size
        out = torch.zeros(shape, dtype=src.dtype, device=src.device)
        return out.index_add_(dim, index, src)

    m.scatter_sum = scatter_sum
    return m


def load_ba_module():
    sys.modules.setdefault("torch_scatter", _make_torch_scatter())
    cuda_ba = types.ModuleType("cuda_ba")

    def _unavailable(*a, **k):
        raise RuntimeError("reference cuda_ba is not built here")

    cuda_ba.neighbors = cuda_ba.reproject = cuda_ba.forward = _unavailable
    sys.modules.setdefault("cuda_ba", cuda_ba)
    sys.modules["lietorch_backends"] = _make_lietorch_backends()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import dpvo.ba as ref_ba  # noqa: E402
    import dpvo.projective_ops as ref_pops  # noqa: E402
    from dpvo.lietorch import SE3  # noqa: E402
    return ref_ba, ref_pops, SE3


# ----------------------------------------------------------------- inputs
def corr_inputs(seed, M, C, N1, N2, H2, W2, p=3, oob_frac=0.2):
    g = torch.Generator().manual_seed(seed)
    fmap1 = 0.25 * torch.randn(1, N1, C, p, p, generator=g)
    fmap2 = 0.25 * torch.randn(1, N2, C, H2, W2, generator=g)
    ii = torch.randint(0, N1, (M,), generator=g)
    jj = torch.randint(0, N2, (M,), generator=g)
    cx = torch.rand(M, 1, 1, generator=g) * (W2 + 8) - 4  # some windows cross the border
    cy = torch.rand(M, 1, 1, generator=g) * (H2 + 8) - 4
    off = torch.arange(p, dtype=torch.float32) - p // 2
    wob = 0.3 * torch.randn(M, 2, p, p, generator=g)  # non-rigid warp of the patch grid
    x = cx + off.view(1, 1, p) + wob[:, 0]
    y = cy + off.view(1, p, 1) + wob[:, 1]
    n_far = int(oob_frac * M)
    if n_far:
        x[:n_far] += 3 * W2  # fully outside
    coords = torch.stack([x, y], 1).unsqueeze(0).contiguous()
    return fmap1, fmap2, coords, ii, jj


def make_corr(cm):
    cases = [
        ("corr_loop_a", dict(seed=1, M=6, C=128, N1=5, N2=3, H2=20, W2=24), 3),
        ("corr_loop_b", dict(seed=2, M=5, C=32, N1=4, N2=2, H2=12, W2=9), 2),
        ("corr_loop_c", dict(seed=3, M=4, C=16, N1=3, N2=2, H2=30, W2=40), 1),
    ]
    for name, kw, R in cases:
        f1, f2, co, ii, jj = corr_inputs(**kw)
        out, = cm.corr_forward_torch_wrapper(f1, f2, co, ii, jj, R)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), fmap1=f1.numpy(), fmap2=f2.numpy(),
                            coords=co.numpy(), ii=ii.numpy(), jj=jj.numpy(), radius=R,
                            out=out.contiguous().numpy())
        print(name, out.shape)
    # grid_sample restatement (fp32), larger edge count
    f1, f2, co, ii, jj = corr_inputs(seed=11, M=64, C=64, N1=24, N2=3, H2=20, W2=28)
    out = cm.corr_torch_forward(f1, f2, co, ii, jj, 3)
    np.savez_compressed(os.path.join(OUT, "corr_gs_a.npz"), fmap1=f1.numpy(), fmap2=f2.numpy(),
                        coords=co.numpy(), ii=ii.numpy(), jj=jj.numpy(), radius=3,
                        out=out.contiguous().numpy())
    print("corr_gs_a", out.shape)


def make_patchify(cm):
    g = torch.Generator().manual_seed(21)
    for name, (C, H, W, M, R) in {"patchify_a": (16, 20, 24, 12, 1), "patchify_b": (8, 9, 11, 7, 0),
                                  "patchify_c": (4, 12, 12, 5, 2)}.items():
        net = torch.randn(1, C, H, W, generator=g)
        coords = torch.stack([torch.rand(1, M, generator=g) * (W + 4) - 2,
                              torch.rand(1, M, generator=g) * (H + 4) - 2], -1)
        zero = cm.patchify_forward_kernel_CPU(R, net, coords)
        clamp = cm.patchify_forward_kernel_python(R, net, coords)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), net=net.numpy(), coords=coords.numpy(),
                            radius=R, out_zero=zero.numpy(), out_clamp=clamp.numpy())
        print(name, zero.shape)


# ----------------------------------------------------------------- BA
def synth_graph(seed, F, M, E, H=120, W=160, p=3, span=5, intr=(80.0, 80.0, 80.0, 60.0),
                noise=0.25, tpad=0, lateral=0.0, wmin=0.0):
    """The SURVEY 8(d) synthetic patch graph recipe (cfg1/cfg2 shaped)."""
    g = torch.Generator().manual_seed(seed)
    oracle_dir = HERE
    sys.path.insert(0, oracle_dir)
    xi = torch.zeros(F, 6, dtype=torch.float64)
    xi[:, 2] = 0.05 * torch.arange(F, dtype=torch.float64)
    xi[:, 0] = lateral * torch.arange(F, dtype=torch.float64)
    xi += 0.01 * torch.randn(F, 6, generator=g, dtype=torch.float64)
    xi[0] = 0
    poses = torch.from_numpy(oracle.lie_fwd(3, "exp", xi.numpy())).float()
    cxy = torch.stack([torch.rand(F * M, generator=g) * (W - 9) + 4,
                       torch.rand(F * M, generator=g) * (H - 9) + 4], -1).floor()
    d = torch.rand(F * M, generator=g) * 1.0 + 0.2
    off = torch.arange(p, dtype=torch.float32) - p // 2
    patches = torch.zeros(F * M, 3, p, p)
    patches[:, 0] = cxy[:, 0].view(-1, 1, 1) + off.view(1, 1, p)
    patches[:, 1] = cxy[:, 1].view(-1, 1, 1) + off.view(1, p, 1)
    patches[:, 2] = d.view(-1, 1, 1)
    # candidate edges (k, j): j in [max(0,i-span), min(F, i+span+1))
    cand = []
    for k in range(F * M):
        i = k // M
        for j in range(max(0, i - span), min(F, i + span + 1)):
            cand.append((k, j))
    cand = torch.tensor(cand)
    # one edge per patch + random extra edges
    first = []
    for k in range(F * M):
        rows = (cand[:, 0] == k).nonzero().view(-1)
        first.append(rows[torch.randint(0, len(rows), (1,), generator=g)].item())
    first = torch.tensor(first)
    mask = torch.ones(len(cand), dtype=torch.bool)
    mask[first] = False
    rest = mask.nonzero().view(-1)
    extra = rest[torch.randperm(len(rest), generator=g)[: max(E - F * M, 0)]]
    sel = torch.cat([first, extra])[:E]
    edges = cand[sel]
    order = torch.argsort(edges[:, 0] * (F + 1) + edges[:, 1])
    edges = edges[order]
    kk = edges[:, 0].long()
    jj = edges[:, 1].long()
    ii = kk // M
    intrinsics = torch.tensor(intr).view(1, 4).repeat(F + tpad, 1)
    coords = torch.from_numpy(oracle.reproject(poses.numpy(), patches.numpy(), intrinsics.numpy(),
                                               ii.numpy(), jj.numpy(), kk.numpy()))
    target = coords[0, :, :, p // 2, p // 2] + noise * torch.randn(len(ii), 2, generator=g)
    weight = wmin + (1 - wmin) * torch.rand(len(ii), 2, generator=g)
    return dict(poses=poses, patches=patches, intrinsics=intrinsics, ii=ii, jj=jj, kk=kk,
                target=target, weight=weight)


def make_ba(ref_ba, ref_pops, SE3):
    for name, (seed, F, M, E) in {"ba_py_a": (31, 6, 8, 96), "ba_py_b": (32, 8, 32, 256)}.items():
        G = synth_graph(seed, F, M, E, lateral=0.1, wmin=0.3, noise=0.1)
        t0 = 1
        t1 = int(max(G["ii"].max(), G["jj"].max())) + 1
        intr = G["intrinsics"][0]
        cx, cy = float(intr[2]), float(intr[3])
        bounds = (-64.0, -64.0, 2 * cx + 64.0, 2 * cy + 64.0)
        poses = SE3(G["poses"].unsqueeze(0).clone())
        patches = G["patches"].unsqueeze(0).clone()
        new_poses, new_patches = ref_ba.BA(
            poses, patches, G["intrinsics"].unsqueeze(0), G["target"].unsqueeze(0),
            G["weight"].unsqueeze(0), 1e-4, G["ii"], G["jj"], G["kk"], bounds, ep=1.0,
            fixedp=t0, structure_only=False)
        # the same reference code in float64 pins the oracle tightly
        p64, k64 = ref_ba.BA(
            SE3(G["poses"].double().unsqueeze(0)), G["patches"].double().unsqueeze(0),
            G["intrinsics"].double().unsqueeze(0), G["target"].double().unsqueeze(0),
            G["weight"].double().unsqueeze(0), 1e-4, G["ii"], G["jj"], G["kk"], bounds, ep=1.0,
            fixedp=t0, structure_only=False)
        dmin, dmax = float(k64[0, :, 2].min()), float(k64[0, :, 2].max())
        # inert-divergence check: ba.py clamps depth to [1e-3, 10], ba_cuda.cu to
        # [1e-4, 20->1]; fixtures must not touch either clamp
        assert 1.01e-3 < dmin and dmax < 9.9, (name, dmin, dmax)
        # reference transform (coords + jacobians) on the same inputs
        coords, valid, (Ji, Jj, Jz) = ref_pops.transform(
            SE3(G["poses"].unsqueeze(0)), G["patches"].unsqueeze(0), G["intrinsics"].unsqueeze(0),
            G["ii"], G["jj"], G["kk"], jacobian=True)
        np.savez_compressed(
            os.path.join(OUT, name + ".npz"), poses=G["poses"].numpy(), patches=G["patches"].numpy(),
            intrinsics=G["intrinsics"].numpy(), ii=G["ii"].numpy(), jj=G["jj"].numpy(),
            kk=G["kk"].numpy(), target=G["target"].numpy(), weight=G["weight"].numpy(), t0=t0,
            t1=t1, lmbda=1e-4, out_poses=new_poses.data[0].numpy(), out_patches=new_patches[0].numpy(),
            out_poses64=p64.data[0].numpy(), out_patches64=k64[0].numpy(),
            tr_coords=coords[0].numpy(), tr_valid=valid[0].numpy(), tr_Ji=Ji[0].numpy(),
            tr_Jj=Jj[0].numpy(), tr_Jz=Jz[0].numpy())
        print(name, "E", len(G["ii"]), "t1", t1)


def load_optim_utils():
    """loop_closure/optim_utils.py with numba / pypose absent: njit runs the
    plain Python function (reduce_edges is pure numpy-style Python)."""
    nb = types.ModuleType("numba")
    nb.bool_ = np.bool_

    def njit(*a, **k):
        if a and callable(a[0]):
            return a[0]
        return lambda f: f

    nb.njit = njit
    sys.modules.setdefault("numba", nb)
    pp = types.ModuleType("pypose")
    pp.__getattr__ = lambda name: type(name, (), {})  # annotations only (pp.SE3, ...)
    sys.modules.setdefault("pypose", pp)
    path = os.path.join(REF, "dpvo", "loop_closure", "optim_utils.py")
    spec = importlib.util.spec_from_file_location("ref_optim_utils", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def loop_scene(seed, N, M, P=3, period=40):
    """a camera circling with `period` frames per lap (revisits -> loop edges)."""
    rng = np.random.default_rng(seed)
    poses = np.zeros((N, 7), np.float32)
    for f in range(N):
        th = 2 * np.pi * f / period
        c = np.array([0.6 * np.sin(th), 0.0, 0.6 * (1 - np.cos(th))])
        ca, sa = np.cos(-th), np.sin(-th)
        Rm = np.array([[ca, 0, sa], [0, 1, 0], [-sa, 0, ca]])
        poses[f, :3] = -Rm @ c + 0.002 * rng.normal(size=3)
        poses[f, 3:] = [0.0, np.sin(-th / 2), 0.0, np.cos(-th / 2)]
    pts = np.zeros((N * M, 3, P, P), np.float32)
    cx, cy = rng.uniform(10, 150, N * M), rng.uniform(10, 110, N * M)
    off = np.arange(P) - P // 2
    pts[:, 0] = cx[:, None, None] + off[None, None, :]
    pts[:, 1] = cy[:, None, None] + off[None, :, None]
    pts[:, 2] = rng.uniform(0.5, 1.5, N * M)[:, None, None]
    intr = np.tile(np.array([100.0, 100.0, 80.0, 60.0], np.float32), (N, 1))
    return poses, pts, intr


def make_keyframe(ref_pops, SE3):
    from einops import reduce

    ou = load_optim_utils()
    M, n, P = 10, 120, 3
    N = n + 8
    poses, pts, intr = loop_scene(71, N, M, P)
    T = torch.from_numpy
    Ps, Ks, Is = SE3(T(poses).unsqueeze(0)), T(pts).unsqueeze(0), T(intr).unsqueeze(0)
    # motionmag input: DPVO-window edges (frames within 3 of each other)
    ei, ej, ek = [], [], []
    for a in range(n - 12, n):
        for b in range(max(0, a - 3), min(n, a + 4)):
            for m in range(M):
                ei.append(a), ej.append(b), ek.append(a * M + m)
    ei, ej, ek = (torch.tensor(v) for v in (ei, ej, ek))
    flow, val = ref_pops.flow_mag(Ps, Ks, Is, ei, ej, ek, beta=0.5)
    # edges_loop (patchgraph.py:74-91), RW 20, GOF 15, KI 4, AGE 1000, thresh 64
    l = n - 20
    jr = torch.arange(n - 15, n - 4)
    kr = torch.arange(max(l - 1000, 0) * M, l * M)
    jj, kk = (t.reshape(-1) for t in torch.meshgrid(jr, kr, indexing="ij"))
    ix = torch.arange(N).repeat_interleave(M)
    ii = ix[kk]
    fmg, lval = ref_pops.flow_mag(Ps, Ks[..., 1, 1].view(1, -1, 3, 1, 1), Is, ii, jj, kk, beta=0.5)
    fsum = reduce(fmg * lval, "1 (fl M) 1 1 -> fl", "sum", M=M).float()
    nval = reduce(lval, "1 (fl M) 1 1 -> fl", "sum", M=M).clamp(min=1)
    fm = torch.where(nval > (M * 0.75), fsum / nval, torch.inf)
    mask = fm < 64.0
    es = ou.reduce_edges(fm[mask].numpy(), ii[::M][mask].numpy(), jj[::M][mask].numpy(),
                         max_num_edges=1000, nms=1)
    edges = torch.as_tensor(es)
    from einops import repeat

    li, lj = repeat(edges, "E ij -> ij E M", M=M, ij=2)
    lk = li.mul(M) + torch.arange(M)
    # reduce_edges on a crafted case: inf, >= 1000, j - i < 30, NMS rows, cap
    rf = np.array([5.0, 1.0, np.inf, 2.0, 1500.0, 3.0, 0.5, 4.0, 2.5, 0.25], np.float32)
    ri = np.array([10, 11, 12, 40, 3, 12, 50, 2, 9, 60], np.int64)
    rj = np.array([60, 60, 60, 90, 60, 61, 70, 61, 60, 95], np.int64)
    res = [ou.reduce_edges(rf, ri, rj, max_num_edges=cap, nms=1) for cap in (1000, 3)]
    np.savez_compressed(
        os.path.join(OUT, "keyframe_a.npz"), poses=poses, patches=pts, intrinsics=intr, M=M, n=n,
        ei=ei.numpy(), ej=ej.numpy(), ek=ek.numpy(), flow=flow[0].numpy(), valid=val[0].numpy(),
        loop_flow=fm.numpy(), loop_kk=lk.flatten().numpy(), loop_jj=lj.flatten().numpy(),
        re_flow=rf, re_ii=ri, re_jj=rj, re_es=res[0], re_es_cap3=res[1])
    print("keyframe_a loop edges", len(es), "flow edges", len(ei))


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(4)
    which = set(sys.argv[1:]) or {"corr", "patchify", "ba", "keyframe"}
    cm = load_corr_module() if which & {"corr", "patchify"} else None
    if "corr" in which:
        make_corr(cm)
    if "patchify" in which:
        make_patchify(cm)
    if which & {"ba", "keyframe"}:
        ref_ba, ref_pops, SE3 = load_ba_module()
        if "ba" in which:
            make_ba(ref_ba, ref_pops, SE3)
        if "keyframe" in which:
            make_keyframe(ref_pops, SE3)


if __name__ == "__main__":
    main()
