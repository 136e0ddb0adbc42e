"""Benchmark: DPVO update iterations/s (altcorr + fastba) on the BASELINE cfg2
synthetic patch graph -- 96 patches x 2048 edges, p=3, 4-level pyramid
[1,2,4,8], fp32 -- on N MI355X GPUs (replicas; one process per GPU).

One step = one DPVO update iteration with all inputs resident in HBM:
  frame     insertion of one new frame into the channels-last pyramid ring
  F-REPROJ  (cuda_ba.reproject, E x 9 points; the same launch inserts the
            frame, orders the edges for A-CORR and plans the BA)
  A-CORR    (all 4 levels in one launch, cuda_corr.forward_levels)
  F-BA      (cuda_ba.forward, 2 iterations, poses/patches updated in place)
By default every kernel is launched from Python each step, as DPVO runs; the
host stays ahead of the GPU (--graph: capture the step once as a hipGraph and
replay it; each replay leaves a ~8.7 us launch gap).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Without a launcher (WORLD_SIZE unset) and N > 1, bench.py starts the N ranks
itself (one child process per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
in each child's environment, before anything touches the GPU) and exits with
the worst child exit code; rank 0 prints the line.

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "update-iterations/sec (altcorr+fastba) on 96-patch/2048-edge graph, 1→8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
TRAFFIC_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                            "profiles", "r06_corr_traffic.json")


def pmc_traffic(config):
    """Per-launch HBM bytes of corr_nhwc_lvl_kernel from the committed PMC passes
    (scripts/pmc.sh + scripts/traffic_summary.py; FETCH_SIZE doubled per the
    gfx950 correction). Counters cannot be read live inside the timed run, so
    the figure is only reported for the default cfg2 workload it was taken on."""
    if config != "cfg2" or not os.path.exists(TRAFFIC_FILE):
        return None
    with open(TRAFFIC_FILE) as f:
        return json.load(f)["traffic_bytes_per_launch"]


def algorithmic_corr_bytes(coords, H2s, W2s, scales, C, p, R, feat_bytes):
    """per edge per level
    B_l = s_f C p^2 (gmap patch) + s_f C U_l (fmap window union) + 2 p^2 4 (coords)
          + 16 (ii, jj) + (2R+1)^2 p^2 4 (output, fp32)
    with U_l = number of distinct in-map fmap pixels touched by the edge's p^2
    windows at level l, computed exactly from the coordinates."""
    import torch

    D = 2 * R + 2
    E = coords.shape[1]
    off = torch.arange(D, device=coords.device) - R
    total = 0
    per_level = []
    for H2, W2, s in zip(H2s, W2s, scales):
        c = coords[0] / s  # [E, 2, p, p]
        x0 = c[:, 0].floor().long().view(E, -1)  # [E, p*p]
        y0 = c[:, 1].floor().long().view(E, -1)
        xs = (x0[:, :, None, None] + off.view(1, 1, 1, D)).expand(E, p * p, D, D)
        ys = (y0[:, :, None, None] + off.view(1, 1, D, 1)).expand(E, p * p, D, D)
        inb = (xs >= 0) & (xs < W2) & (ys >= 0) & (ys < H2)
        key = torch.where(inb, ys * W2 + xs, torch.full_like(xs, -1)).reshape(E, -1)
        key, _ = key.sort(dim=1)
        distinct = ((key[:, 1:] != key[:, :-1]) & (key[:, 1:] >= 0)).sum(1) + (key[:, 0] >= 0).long()
        U = distinct.sum().item()
        b = E * (feat_bytes * C * p * p + 2 * p * p * 4 + 16 + (2 * R + 1) ** 2 * p * p * 4)
        b += feat_bytes * C * U
        per_level.append({"scale": s, "U_mean": U / E, "bytes": b})
        total += b
    return total, per_level


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n, port, base=None):
    """Environment of each of the n ranks bench.py starts itself (the same
    variables torch.distributed.run sets)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                  "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(port), "DPVO_BENCH_CHILD": "1"})
        # RCCL / CUDA-tensor IPC on this host needs dmabuf (see the environment notes)
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        envs.append(e)
    return envs


def launch_ranks(n, argv, cmd=None):
    """Run `cmd` (default: this script with `argv`) as n rank processes and
    return the worst exit code.  Called only when WORLD_SIZE is unset: nothing
    in this parent process has touched the GPU (no torch import at all)."""
    import subprocess

    cmd = cmd or [sys.executable, os.path.abspath(__file__), *argv]
    procs = [subprocess.Popen(cmd, env=e) for e in rank_envs(n, free_port())]
    # poll: a rank that fails (e.g. before or inside init_process_group) ends the
    # run at once instead of leaving the others in rendezvous until its timeout
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc is not None and rc != 0]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(rc is not None for rc in rcs):
            return 0
        time.sleep(0.05)


def warm_until(step_fn, torch, min_ms=200.0, max_steps=100000):
    """Run steps until at least min_ms of wall time has passed (GPU clocks
    ramp on a fresh box; a fixed step count can end before they have)."""
    t0 = time.perf_counter()
    n = 0
    while n < max_steps:
        for _ in range(8):
            step_fn(n)
            n += 1
        torch.cuda.synchronize()
        if (time.perf_counter() - t0) * 1e3 >= min_ms:
            break
    return n


def sharded_main(args, torch, dist, world, rank, local, dev):
    """--sharded: BASELINE cfg4 global BA (1024 frames x 96 patches, ~131k
    edges, N = 1023 free poses), edge-sharded by source frame over the ranks
    with ONE RCCL all_reduce(SUM) of the packed fp64 (y, S blocks) per BA
    iteration (dpvo_amd/fastba/sharded.py).  A step = one global
    BA call (setup + iterations), as __run_global_BA issues it
    (dpvo.py:695-715).  Reports us per BA iteration, all-reduce bytes and the
    all-reduce share of the iteration time (rank 0's HIP events)."""
    from dpvo_amd import synthetic
    from dpvo_amd.fastba.sharded import ShardedBA

    G = synthetic.make_config(args.config if args.config != "cfg2" else "cfg4", seed=args.seed)
    D = G.to(dev)
    t0, t1 = 1, G.F
    lmbda = torch.tensor([1e-4], device=dev)
    poses0, patches0 = D.poses.clone(), D.patches.clone()
    group = dist.group.WORLD if world > 1 else None

    def step():
        poses, patches = poses0.clone(), patches0.clone()
        sb = ShardedBA(D.ii, D.jj, D.kk, patches.shape[0], G.M, t0, t1, group=group)
        sb(poses, patches, D.intrinsics, D.target, D.weight, lmbda, iterations=args.ba_iters)
        return sb, poses

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    warm_until(lambda i: step(), torch, args.warm_ms)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    tt = time.perf_counter()
    for _ in range(args.steps):
        sb, poses = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - tt
    # phase split of one iteration on this rank: build | all_reduce | solve+update
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    poses, patches = poses0.clone(), patches0.clone()
    st = sb.state
    reps = max(3, min(args.steps, 10))
    acc = [0.0, 0.0, 0.0]
    for _ in range(reps):
        ev[0].record()
        sb.backend.build(st, poses, patches, D.intrinsics, D.target, D.weight, lmbda, D.ii, D.jj)
        ev[1].record()
        if world > 1:
            dist.all_reduce(sb.backend.packed(st), op=dist.ReduceOp.SUM, group=group)
        ev[2].record()
        sb.backend.solve_update(st, poses, patches)
        ev[3].record()
        torch.cuda.synchronize()
        for k in range(3):
            acc[k] += ev[k].elapsed_time(ev[k + 1]) / reps
    info = sb.backend.status(st)
    status = info[0]
    if world > 1:
        t = torch.tensor([elapsed] + acc, device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, acc = t[0].item(), t[1:].tolist()
    it_ms = sum(acc)
    if rank == 0:
        out = {
            "metric": "global-BA iterations/s (cfg4 sharded fastba, eff_impl)",
            "value": args.steps * args.ba_iters / elapsed,
            "unit": "BA-iterations/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32 edge math, f64 S/solve",
            "data": "synthetic (SURVEY 8d cfg4 recipe, seeded)",
            "config": {"workload": f"{args.config if args.config != 'cfg2' else 'cfg4'}: "
                                   f"{G.F} frames x {G.M} patches, {G.E} edges, N={t1 - t0}, "
                                   f"BA {args.ba_iters} iters per call (setup included)",
                       "edges": G.E, "frames": G.F, "parallelism": f"edge-sharded x{world}"},
            "per_iteration_ms": {"build": acc[0], "all_reduce": acc[1], "solve_update": acc[2],
                                 "total": it_ms},
            "all_reduce_bytes": sb.allreduce_bytes,
            "all_reduce_share": acc[1] / it_ms if it_ms > 0 else 0.0,
            "ba_status": status,
            "structure": dict(zip(["status", "patches", "items", "blocks", "interior", "border",
                                   "g", "superblocks"], info)),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--levels", default="1,2,4,8")
    ap.add_argument("--ba-iters", type=int, default=2)
    ap.add_argument("--mem", type=int, default=36, help="feature ring-buffer frames (DPVO mem)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--overlap", action="store_true",
                    help="issue the BA edge grouping (fastba.plan) on a side stream "
                         "concurrently with A-CORR.  Off by default: in the replayed graph the "
                         "cross-queue join before the BA costs ~11 us, more than the 12 us "
                         "plan kernel it hides (profiles/r02_trace_overlap_vs_inline.txt)")
    ap.add_argument("--separate-plan", action="store_true",
                    help="launch the BA edge grouping as its own kernel after A-CORR (default: "
                         "inside the reprojection launch, fastba.reproject(plan_window=...))")
    ap.add_argument("--separate-insert", action="store_true",
                    help="insert the frame into the pyramid as its own launch (default: inside "
                         "the reprojection + plan launch, on the CUs those leave idle)")
    ap.add_argument("--sharded", action="store_true",
                    help="cfg4 global BA, edge-sharded over the ranks (one RCCL all_reduce of "
                         "the packed (S, y) per iteration); --config picks the large graph")
    ap.add_argument("--features", choices=["f32", "f16"], default="f32",
                    help="feature dtype of the pyramid / gmap rings (f16 = the fork's "
                         "MIXED_PRECISION runtime: A-CORR on v_mfma_f32_16x16x16_f16)")
    ap.add_argument("--warm-ms", type=float, default=200.0,
                    help="after the --warmup steps, keep stepping (untimed) until this much wall "
                         "time has passed: clocks ramp on a fresh box")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as one captured hipGraph (default: launch every kernel "
                         "from Python each step, as DPVO does; the host stays ahead of the GPU, "
                         "while a graph replay leaves a ~8.7 us gap between steps: "
                         "profiles/r02_trace_overlap_vs_inline.txt)")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # --gpus N without a launcher: start the N ranks here (before any GPU call)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE = {world}")
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
    dev = torch.device("cuda", local)
    if args.sharded:
        return sharded_main(args, torch, dist, world, rank, local, dev)

    from dpvo_amd import altcorr, fastba, synthetic

    levels = [int(x) for x in args.levels.split(",")]
    G = synthetic.make_config(args.config, seed=args.seed)  # same graph on every rank (replicas)
    D = G.to(dev)
    P = G.patches.shape[-1]
    C = 128
    # the network emits NCHW features; the ring buffer keeps them channels-last
    # (corr_nhwc.hip).  Every step inserts one frame (NCHW level 1 -> pooled,
    # channels-last levels, one launch) so the per-frame cost of the pyramid and
    # its layout is inside the timed region.
    fdt = torch.float16 if args.features == "f16" else torch.float32
    feat_bytes = 2 if args.features == "f16" else 4
    pyr_nchw = synthetic.make_features(mem=args.mem, C=C, levels=levels, seed=args.seed,
                                       device=dev, dtype=fdt)
    pyr = [synthetic.channels_last(p) for p in pyr_nchw]
    # gmap: patch features of every (frame, slot), DPVO's pmem = mem ring
    gbuf = torch.zeros(1, args.mem * G.M, C, P, P, device=dev, dtype=fdt)
    centres = D.patches[: G.F * G.M, :2, P // 2, P // 2]  # [F*M, 2] (x, y)
    for f in range(G.F):
        gbuf[0, f * G.M:(f + 1) * G.M] = altcorr.patchify(
            pyr_nchw[0][:, f], centres[f * G.M:(f + 1) * G.M].unsqueeze(0), P // 2)[0]
    lmbda = torch.tensor([1e-4], device=dev)
    poses, patches = D.poses.clone(), D.patches.clone()
    kk1 = D.kk % (G.M * args.mem)  # dpvo.py:456-457
    jj1 = D.jj % args.mem
    scales = [float(s) for s in levels]

    plan_stream = torch.cuda.Stream()
    fused_plan = (not args.overlap and not args.separate_plan
                  and fastba.cuda_ba.plan_supported(int(D.ii.numel()), 1, G.F, P))
    fused_insert = fused_plan and not args.separate_insert

    def step(i=0, ev=None):
        cur = torch.cuda.current_stream()
        ws = None
        if args.overlap:
            # the BA edge grouping reads the patch graph only (fixed before the
            # update, dpvo.py:775-824): issue it on a side stream so it runs
            # concurrently with the frame insertion / reprojection / A-CORR
            plan_stream.wait_stream(cur)
            with torch.cuda.stream(plan_stream):
                ws = fastba.plan(D.ii, D.jj, D.kk, 1, G.F, patches.shape[0], poses.shape[0], P)
            if ws is not None:
                ws.record_stream(cur)
        slot = i % args.mem  # frame insertion (dpvo.py:__call__ -> ring buffer)
        if fused_insert:
            # frame insertion + reprojection + A-CORR edge order + BA plan, one launch
            coords, order, ws = fastba.reproject(
                poses, patches, D.intrinsics, D.ii, D.jj, D.kk, mem=args.mem, plan_window=(1, G.F),
                insert=(pyr_nchw[0][0, slot], [p[0, slot] for p in pyr], levels))
        else:
            altcorr.insert_frame(pyr_nchw[0][0, slot], pyr, slot, levels)
        # reprojection + the XCD-aware edge order (edges grouped by target
        # frame) in one launch; A-CORR processes each group on one XCD
        if fused_insert:
            pass
        elif fused_plan:
            # ... and the BA edge grouping (reads ii / jj / kk only, fixed for
            # the update) as workgroup 0 of the same launch
            coords, order, ws = fastba.reproject(poses, patches, D.intrinsics, D.ii, D.jj, D.kk,
                                                 mem=args.mem, plan_window=(1, G.F))
        else:
            coords, order = fastba.reproject(poses, patches, D.intrinsics, D.ii, D.jj, D.kk,
                                             mem=args.mem)
        if ev is not None:
            ev[0].record()
        corr = altcorr.corr_levels(gbuf, pyr, coords, kk1, jj1, 3, scales, order=order)
        if ev is not None:
            ev[1].record()
        if args.overlap:
            cur.wait_stream(plan_stream)
        fastba.BA(poses, patches, D.intrinsics, D.target, D.weight, lmbda, D.ii, D.jj, D.kk, 1,
                  G.F, M=G.M, iterations=args.ba_iters, plan=ws)
        return corr

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    warm_until(step, torch, args.warm_ms)
    # A-CORR kernel time for the roofline: HIP events around the corr launch
    # (same stream) over eager steps outside the timed region
    n_ev = 20
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(n_ev)]
    for i in range(n_ev):
        step(i, evs[i])
    torch.cuda.synchronize()
    corr_ms = sorted(a.elapsed_time(b) for a, b in evs)[n_ev // 2]
    coords0 = fastba.reproject(poses, patches, D.intrinsics, D.ii, D.jj, D.kk)
    alg_bytes, per_level = algorithmic_corr_bytes(
        coords0, [f.shape[3] for f in pyr], [f.shape[4] for f in pyr], scales, C, P, 3,
        feat_bytes)

    graph = None
    if args.graph:
        # one update iteration (frame insertion, reproject, corr, 2 BA iterations)
        # captured once and replayed: the same kernels with the same work, without
        # the per-launch Python / runtime gaps
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for i in range(3):
                step(i)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step(0)
        graph.replay()
        torch.cuda.synchronize()

    # The host call of the first timed step used to take ~0.22 ms (against
    # ~0.03 ms for the others; step_split.host_enqueue_ms_first) with the GPU
    # idle meanwhile -- 7 % of a 20-step run, the driver-vs-long-run gap of
    # VERDICT r04 weak 2.  The roofline bookkeeping above (torch sorts, .item()
    # syncs, fresh Python objects) ran right before it; now a garbage
    # collection and a second (short) time-based warm-up come last.
    gc.collect()
    warm_until(step if graph is None else (lambda i: graph.replay()), torch,
               min(50.0, args.warm_ms))

    def run_one(i):
        if graph is not None:
            graph.replay()
        else:
            step(i)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    host_s = [0.0] * args.steps
    t0 = time.perf_counter()
    for i in range(args.steps):
        h = time.perf_counter()
        run_one(i)
        host_s[i] = time.perf_counter() - h  # host enqueue time of the step (no sync)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # per-step split, in a second pass of the same length
    # right after the timed one (events are not recorded inside the timed loop):
    # HIP events before / after each step on the launch stream = the GPU time
    # of the step's kernels incl. the gaps between them; host enqueue = the
    # wall time of the Python call (perf_counter, no sync) in the timed loop
    n_pp = max(args.steps, 20)
    pev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(n_pp)]
    for i in range(n_pp):
        pev[i][0].record()
        run_one(i)
        pev[i][1].record()
    torch.cuda.synchronize()
    gpu_ms = sorted(a.elapsed_time(b) for a, b in pev)
    host_ms = sorted(1e3 * h for h in host_s)
    step_split = {
        "gpu_ms_median": gpu_ms[n_pp // 2], "gpu_ms_min": gpu_ms[0], "gpu_ms_max": gpu_ms[-1],
        "host_enqueue_ms_median": host_ms[len(host_ms) // 2], "host_enqueue_ms_max": host_ms[-1],
        "host_enqueue_ms_first": 1e3 * host_s[0],
        "note": "gpu = HIP events around each step (second pass, same length); host = "
                "perf_counter around each timed step() call without a sync",
    }

    # every BA call of the run (warmup, event steps, graph replays) finished
    # without a fatal status (raises RuntimeError otherwise)
    ba_status = fastba.cuda_ba.check_status(poses)

    per_rank = [args.steps / elapsed]
    if world > 1:
        mine = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        allt = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allt, mine)
        per_rank = [args.steps / t.item() for t in allt]
        t = torch.tensor([elapsed, corr_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, corr_ms = t[0].item(), t[1].item()

    value = world * args.steps / elapsed
    achieved = alg_bytes / (corr_ms * 1e-3) / 1e9  # GB/s of the dominant kernel

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import cpu_baseline  # baseline infrastructure (CPU port of the reference path)

        # all cores of this process's share of the host (16 on the GPU box;
        # os.cpu_count() shows the whole machine there), then the 2 threads
        # DPVO.__init__ sets (dpvo.py:66), then the fork's 1-iteration local BA
        threads = min(16, os.cpu_count() or 1)
        kw = dict(levels=tuple(levels), mem=args.mem, C=C)
        ips, thr, n = cpu_baseline.measure(G, budget_s=args.cpu_budget, threads=threads,
                                           iterations=args.ba_iters, **kw)
        ips2, thr2, n2 = cpu_baseline.measure(G, budget_s=args.cpu_budget, threads=2,
                                              iterations=args.ba_iters, **kw)
        ips1, thr1, n1 = cpu_baseline.measure(G, budget_s=0.5 * args.cpu_budget, threads=threads,
                                              iterations=1, **kw)
        cpu = {"value": ips, "unit": "update-iterations/s", "cores": thr, "kind": "port",
               "sample": f"{n} full {args.config} update iteration(s) (reproject + "
                         f"{len(levels)}-level grid_sample corr + {args.ba_iters} ba.py BA "
                         f"steps), torch CPU, {thr} threads",
               "os_cpu_count": os.cpu_count(),
               "two_threads": {"value": ips2, "cores": thr2, "sample": f"{n2} iteration(s)"},
               "ba_iterations_1": {"value": ips1, "cores": thr1, "sample": f"{n1} iteration(s)"},
               "calibration": "port == reference corr_torch_forward bit for bit, time ratio "
                              "0.96-1.01 (profiles/r02_cpu_calibration.json); ba.py port pinned "
                              "to the reference's fp64 run (tests/test_cpu_baseline.py)"}

    if rank == 0:
        traffic = pmc_traffic(args.config) if args.features == "f32" else None
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "update-iterations/s",
            "n_gpus": world,
            "world_size": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "per_rank_value": per_rank,
            "steps": args.steps,
            "warmup": args.warmup,
            "warm_ms": args.warm_ms,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "step_split": step_split,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.features == "f32" else "f16 features, f32 accumulate",
            "data": "synthetic (SURVEY 8d cfg2 recipe, seeded)",
            "launch": "eager" if graph is None else "hipGraph replay of one captured step",
            "ba_plan": ("side stream, concurrent with A-CORR" if args.overlap else
                        "in the reprojection launch" if fused_plan else "inline (same stream)"),
            "frame_insertion": ("in the reprojection + plan launch" if fused_insert else
                                "own launch"),
            "config": {
                "workload": f"{args.config}: {G.M} patches/frame x {G.E} edges, p={P}, "
                            f"{len(levels)}-level pyramid {levels}, "
                            f"{'fp32' if args.features == 'f32' else 'fp16'} features, "
                            f"BA {args.ba_iters} iters",
                "patches_per_frame": G.M, "edges": G.E, "frames": G.F, "levels": levels,
                "radius": 3, "channels": C, "feature_ring": args.mem,
                "parallelism": f"replicas x{world}",
            },
            "roofline": {
                "kernel": "corr_nhwc_lvl_kernel (A-CORR, all levels, one launch, one wave per "
                          "(edge, level))",
                # how the products are formed (exact fp32 for fp32 features)
                "products": ("fp32 x fp32 on v_mfma_f32_16x16x4_f32 (IEEE fp32 products), fp32 "
                             "accumulation"
                             if args.features == "f32" else
                             "fp16 x fp16 on v_mfma_f32_16x16x32_f16, fp32 accumulation"),
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                # counter (real DRAM) rate of the same launch: PMC bytes / the
                # live kernel time; below `achieved` because edges sharing a
                # target frame re-read overlapping boxes from L2 / MALL
                "traffic_gbs": (traffic / (corr_ms * 1e-3) / 1e9) if traffic else None,
                # the same as a fraction of the peak: `frac` counts every byte the
                # kernel's loads request (the survey's per-edge count), re-reads
                # served by L2 / MALL included, so it can exceed 1
                "traffic_frac": (traffic / (corr_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                "algorithmic_bytes_per_launch": alg_bytes,
                "kernel_ms": corr_ms,
                "per_level": per_level,
            },
            "cpu_baseline": cpu,
            "ba_status": ba_status,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
