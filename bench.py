#!/usr/bin/env python3
"""Headline benchmark: train iters/sec + forward Mpix/sec, 1M Gaussians @ 1920x1080, SH degree 3
(BASELINE.json metric; configs[2] at N=1, configs[3] view-sharded at N>1).

    python bench.py --gpus N --steps K --warmup W
    (N>1 under a launcher: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr
     127.0.0.1 ... bench.py --gpus N ...; WORLD_SIZE must equal --gpus.  N>1 without one: bench.py starts
     that launcher itself as a child process, before anything touches the GPU, and exits with its code)

A "step" is one iteration of the reference's train.py loop (train.py:71-147) on every rank:
lr update, render forward, L1+SSIM loss, backward through the MI355X rasterizer, (gradient
exchange), densification statistics, densify/prune at every multiple of 100, Adam.  Iteration
numbers (they drive the lr schedule and the densify/prune events, train.py:136-143):
  warmup   W iterations ending on densify iteration 900 (allocator and densify path warm)
  profile  901 .. 900+PW: every stage event-timed (the per-kernel breakdown)
  999, 1000  each run alone between device syncs: an ordinary and a densify/prune iteration
           (densify_iter_ms, densify_extra_ms)
  timed    1001 .. 1000+K: it starts right after a densify iteration, so it holds exactly
           floor(K/100) densify/prune events (iterations 1100, 1200, ...) — the reference's
           1-in-100 share, rounded down; `iters_per_s_1in100` adds the measured extra cost of one
           densify iteration per 100 to the ordinary steps of a window without one.
value = iterations all ranks completed in the timed window / wall time (max over ranks).

Data: synthetic and seeded (no datasets offline) — 1M random Gaussians (SURVEY §8(d) bench
variant), 200 Fibonacci-sphere cameras, ground-truth images rendered from a second random model.

Extra objects on the JSON line:
  roofline      heaviest HBM-bound kernel of the step (HIP events on the launch stream), algorithmic
                bytes per launch from SURVEY §8(d) x the frame's measured L / V / L_eff / T / N;
                the VALU-bound blends beside it (blend_fwd / blend_bwd) and the heaviest kernel
                overall (step_dominant)
  cpu_baseline  the CPU oracle (oracle/raster_oracle.c, "port") on the same frame, timed on rank 0
                at every N (--no-cpu-baseline skips it)
  sync_loss_*   the timed step with the reference's per-iteration `loss.item()` read-back (train.py:120)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
VALU_PEAK_TFLOPS = 157.3


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU).  N > 1 without a torch.distributed.run environment: this "
                        "process starts `python -m torch.distributed.run --nproc-per-node N ... bench.py` as "
                        "a child and exits with its code; under a launcher it must equal WORLD_SIZE")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--points", type=int, default=1_000_000)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--views", type=int, default=200)
    p.add_argument("--sh-degree", type=int, default=3)
    p.add_argument("--fwd-frames", type=int, default=50)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--no-profile", action="store_true", help="skip HIP-event stage timing in the timed region")
    p.add_argument("--aux-normal", action="store_true",
                   help="forward-only leg renders the aux depth + normal outputs (BASELINE configs[4] stress)")
    p.add_argument("--binning-split", type=int, default=0,
                   help="early-stop binning: phase A = 1/N of the pairs (1 = one phase; 0 = library default)")
    p.add_argument("--force-dist", action="store_true",
                   help="init the RCCL process group and run the sharded exchange path even at world 1 "
                        "(rehearses the multi-GPU code path on one GPU; not the headline configuration)")
    p.add_argument("--sync-loss-steps", type=int, default=20,
                   help="steps of the extra leg that reads the loss back every iteration (train.py:120)")
    return p.parse_args(argv)


def launch_plan(gpus, env, force_dist=False):
    """What this invocation does with `--gpus`: ("run", world) runs the benchmark in this process as
    one rank of `world`; ("spawn", n) starts n ranks through torch.distributed.run as a child process;
    ("error", msg) refuses.  Pure (no torch, no GPU), so the parent of a spawn never touches the GPU
    before the ranks do (an exec from a GPU-initialised process is forbidden on the box, and a
    parent holding the device would count against the box's per-card process limit).
    force_dist: the one-rank process group needs the launcher's environment too (RANK, MASTER_*),
    so a forced exchange without a launcher spawns one rank."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        try:
            world = int(ws)
        except ValueError:
            return ("error", f"WORLD_SIZE={ws!r} is not an integer")
        if gpus is not None and gpus != world:
            return ("error", f"--gpus {gpus} does not match WORLD_SIZE={world} from the launcher")
        return ("run", world)
    n = 1 if gpus is None else gpus
    if n < 1:
        return ("error", f"--gpus {n}: need at least one GPU")
    return ("spawn", n) if n > 1 or force_dist else ("run", 1)


def spawn_command(n, argv, port, script=None):
    """The child command line of a spawn: one rank per GPU on this node, rendezvous on 127.0.0.1,
    bench.py with the same arguments (WORLD_SIZE from the launcher then equals --gpus)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", script or os.path.join(ROOT, "bench.py"), *argv]


def _spawn(n, argv, script=None):
    """Run the N ranks as a child process (subprocess, not exec), its stdout / stderr inherited, so
    rank 0's JSON line is this process's output; a SIGTERM / SIGINT to this process is passed on."""
    import signal
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    child = subprocess.Popen(spawn_command(n, argv, port, script), env=env)

    def forward(sig, _frame):
        child.send_signal(sig)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    return child.wait()


MODELED = ("preprocess", "scan", "duplicate", "tile_sort", "ranges", "blend_fwd", "blend_bwd", "gauss_bwd")
VALU_BOUND = ("blend_fwd", "blend_bwd")


def algorithmic_bytes(stage, st, P, W, H, K, world=1, sharded=None):
    """SURVEY §8(d) algorithmic bytes per frame (one training step renders one frame).  Binning
    stages are priced on the (bin, Gaussian) pairs this implementation actually sorts (num_binned:
    bins of 2 x 2 tiles, after exact culling and early-stop binning), not on the reference's larger
    num_rendered, so they are not credited for pairs they never write.  The bin sort ("tile_sort")
    is priced at its minimum: read + write each key and u32 value once; the expand ("ranges") at
    reading the sorted pairs once and gathering each pair's 4-B depth key for the per-bin depth sort
    (rr_bin.hip k_sortexpand; its per-tile list writes are not counted)."""
    Lb, V, Le, T, N = st["num_binned"], st["num_visible"], st["l_eff"], st["tiles"], W * H
    M = K
    kw = 2 if (W + 31) // 32 * ((H + 31) // 32) <= 65536 else 4
    return {
        "preprocess": 20 * P + V * (99 + 12 * K),
        "scan": 8 * P,
        "duplicate": 4 * P + 16 * V + (kw + 4) * Lb,
        "tile_sort": 2 * (kw + 4) * Lb,
        "ranges": (kw + 8) * Lb + 8 * T,
        "blend_fwd": 8 * T + 44 * Le + 24 * N,
        "blend_bwd": 8 * T + 40 * Le + 20 * N + 44 * V,
        "gauss_bwd": (gauss_bwd_views_bytes(P, K, M, world) if (world > 1 if sharded is None else sharded)
                      else gauss_bwd_bytes(P, V, K, M, next_frame=st.get("next_frame", False))),
    }.get(stage)


def gauss_bwd_views_bytes(P, K, M, world):
    """The Gaussian-sharded step's per-Gaussian backward on one rank (rain_amd/sharded.py): its
    P/N rows' parameters and both moments read and written once (Adam), statistics read + written,
    and one 40-B record per row and view."""
    rows = (P + world - 1) // world
    return rows * (24 * (11 + 3 * M) + 24) + 40 * rows * world


def gauss_bwd_bytes(P, V, K, M, fused_adam=True, next_frame=False):
    """Per-Gaussian backward.  In the training step (fused_adam) it reads the 64-B gradient
    accumulator line and applies Adam in place: read + write of parameter, exp_avg and exp_avg_sq
    (n_par = 11 + 3M floats each: xyz 3, f_dc 3, f_rest 3(M-1), opacity 1, scaling 3, rotation 4),
    plus the densification statistics of visible Gaussians (read + write of 3 floats).  With the
    next frame's preprocess in the same pass (rr_next_frame) it also writes that frame's geometry:
    radius, pair counts and depth key of every Gaussian (16 B) and the 48-B splat record of the
    visible ones (V of the next frame, taken as this frame's).  The reference-API backward instead
    zero-fills and writes its gradient tensors."""
    if fused_adam:
        return 64 * P + 24 * (11 + 3 * M) * P + 24 * V + ((16 * P + 48 * V) if next_frame else 0)
    return 4 * P * (27 + 3 * M) + 4 * P + 88 * V + 4 * P + V * (143 + 24 * K)


def main():
    args = parse()
    what, val = launch_plan(args.gpus, os.environ, args.force_dist)
    if what == "error":
        print(f"bench.py: {val}", file=sys.stderr)
        return 2
    if what == "spawn":
        rc = _spawn(val, sys.argv[1:])
        return rc if rc >= 0 else 128 - rc
    # The JSON line is the only thing on stdout: native libraries' banners (RCCL prints its version
    # block at communicator creation) go to stderr with everything else.
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    import numpy as np
    import torch
    import torch.distributed as dist

    world = val
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    force = args.force_dist
    if world > 1 or force:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.manual_seed(0)
    np.random.seed(0)

    from rain_amd import _native, synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.diff_gaussian_rasterization import _C
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams
    from rain_amd.renderer import PipelineParams, render, render_depth_normal
    from rain_amd.train import TrainConfig, Trainer

    P, W, H, D = args.points, args.width, args.height, args.sh_degree
    if args.binning_split:
        _native.check(_native.raster().rr_set_binning_config(args.binning_split, 0), "binning config")
    cams = [c.to(dev) for c in fibonacci_cameras(args.views, W, H)]
    extent = 4.0 * 1.1  # getNerfppNorm of the camera rig (dataset_readers.py:34-55): radius 4, x1.1

    # ground truth: a second random model rendered from every view
    gt_model = GaussianModel(D, device=dev)
    gt_model.set_params(synthetic.random_gaussians(P, sh_degree=D, seed=1, bench=True, device=dev))
    gt_model.active_sh_degree = D
    pipe = PipelineParams()
    bg = torch.zeros(3, device=dev)
    with torch.no_grad():
        gts = [render(c, gt_model, pipe, bg)["render"].clamp(0.0, 1.0).contiguous() for c in cams]
    del gt_model

    gauss = GaussianModel(D, divide_ratio=0.8, device=dev)
    gauss.set_params(synthetic.random_gaussians(P, sh_degree=D, seed=0, bench=True, device=dev))
    gauss.active_sh_degree = D
    gauss.spatial_lr_scale = extent
    opt = OptimizationParams()
    gauss.training_setup(opt)
    trainer = Trainer(gauss, cams, gts, opt, pipe, TrainConfig(seed=0), scene_extent=extent,
                      exchange=True if force else None)

    K, Wm = args.steps, args.warmup
    prof = not args.no_profile
    # untimed per-stage breakdown window (every stage event-timed) between warmup and the timed loop
    PW = min(20, K) if prof else 0
    D0, D1 = 900, 1000  # densify/prune iterations (train.py:136-140: multiples of 100 in (500, 15000))
    for it in range(D0 - Wm + 1, D0 + 1):
        trainer.step(it)
    it = D0 + 1
    breakdown, dom, step_dom = {}, None, None
    if prof:
        _native.Profiler.collect()  # drop anything recorded before the window
        with _native.Profiler():
            for _ in range(PW):
                trainer.step(it)
                it += 1
        breakdown = _native.Profiler.collect()
        modeled = [k for k in breakdown if breakdown[k][1] and k in MODELED]
        # the roofline object is priced in HBM bytes: it reports the heaviest kernel whose bound is
        # HBM.  The two blends are VALU-issue bound by construction (44 B per pair
        # against 256 pixel evaluations) and are reported beside it (roofline.blend_fwd / blend_bwd,
        # with their VALU fractions); step_dominant names the heaviest kernel overall.
        step_dom = max(modeled, key=lambda k: breakdown[k][0]) if modeled else None
        hbm_bound = [k for k in modeled if k not in VALU_BOUND]
        dom = max(hbm_bound, key=lambda k: breakdown[k][0]) if hbm_bound else step_dom
    # one ordinary and one densify/prune iteration, each alone between device syncs
    one_ms = {}
    for it in (D1 - 1, D1):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        info = trainer.step(it)
        torch.cuda.synchronize()
        one_ms[it] = 1000.0 * (time.perf_counter() - t0)
    assert info.densified, "iteration 1000 must densify"
    if world > 1:
        e = torch.tensor([one_ms[D1 - 1], one_ms[D1]], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        one_ms = {D1 - 1: float(e[0]), D1: float(e[1])}
    it = D1 + 1
    start_iter = it
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timer = _native.Profiler([dom]) if dom else None
    if timer:  # the timed loop records only the reported kernel: two events per launch
        timer.__enter__()
    # trace markers around the timed loop, outside its clock: a rocprofv3 kernel trace of this run
    # is cut to exactly these K steps by tools/step_breakdown.py --window (profiles/*_timed_*)
    mark = _native.train_lib().rt_trace_marker
    _native.check_rt(mark(0, K, _native.stream_of(trainer.background)), "trace marker")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    views_used = []
    for _ in range(K):
        info = trainer.step(it)
        views_used.append(info.view)
        it += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    _native.check_rt(mark(1, K, _native.stream_of(trainer.background)), "trace marker")
    dom_timed = None
    if timer:
        timer.__exit__()
        dom_timed = _native.Profiler.collect()[dom]
    elapsed = t1 - t0
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    iters_per_s = world * K / elapsed
    ms_per_step = 1000.0 * elapsed / K
    # the Gaussian-sharded step keeps parameters current on their owner's rows only: gather full
    # replicas for the measurement legs below (no-op at world 1)
    trainer.sync_state()
    end_iter = it - 1
    n_densify = sum(1 for i in range(start_iter, end_iter + 1) if i % 100 == 0)
    densify_extra_ms = one_ms[D1] - one_ms[D1 - 1]
    # the reference's share (1 densify/prune iteration in 100) on top of the measured steps
    ms_1in100 = ms_per_step + densify_extra_ms / 100.0 if n_densify == 0 else ms_per_step

    # the same step with the reference's per-iteration loss read-back (train.py:120 `loss.item()`,
    # a device -> host sync every iteration), which the timed loop leaves out: its cost, measured
    sync_it0 = _clear_window(end_iter + 1, 3 + args.sync_loss_steps)
    sync_ms = _timed_steps(trainer, sync_it0, args.sync_loss_steps, world, dev, sync_loss=True)
    sync_end = sync_it0 + 3 + args.sync_loss_steps - 1

    # the reference's own timing bracket (train.py:71-117: iter_start before render, iter_end after
    # loss.backward()): render forward + L1/SSIM + backward, no optimizer step, no densification
    bracket_ms = _bracket(trainer, cams, gts, K if K < 50 else 50, world, dev)
    # the RAIN-GS coarse-to-fine stress regime (train.py:95-107): the same bracket with the 2-D
    # dilation the schedule applies early in training (up to c2f_max_lowpass = 300 px^2; radii of
    # 52+ px and several times the pairs per frame)
    c2f_ms = {str(lp): round(_bracket(trainer, cams, gts, 5, world, dev, low_pass=lp), 3) for lp in (30.0, 300.0)}

    # the same iteration through the reference's own API (what an unchanged train.py:109-147 runs):
    # render() -> GaussianRasterizer autograd -> getters' autograd -> torch.optim.Adam
    api_it0 = (sync_end // 100 + 1) * 100 + 1
    api_ms = _api_leg(gauss, cams, gts, opt, pipe, extent, api_it0, K if K < 30 else 30, world, dev,
                      torch_adam=False)
    api_ta_ms = _api_leg(gauss, cams, gts, opt, pipe, extent, api_it0 + 40, K if K < 30 else 30, world, dev)

    # forward-only throughput (preprocess -> blend incl. sorts and the L read-back), no autograd
    Pn = gauss.get_xyz.shape[0]
    with torch.no_grad():
        for i in range(3):
            render(cams[i], gauss, pipe, bg)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tf0 = time.perf_counter()
        for i in range(args.fwd_frames):
            if args.aux_normal:
                render_depth_normal(cams[(rank * 7 + i) % len(cams)], gauss, bg)
            else:
                render(cams[(rank * 7 + i) % len(cams)], gauss, pipe, bg)
        torch.cuda.synchronize()
        tf = time.perf_counter() - tf0
    if world > 1:
        e = torch.tensor([tf], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        tf = float(e.item())
    fwd_mpix = world * args.fwd_frames * W * H / tf / 1e6

    # frame statistics for the algorithmic-byte model (re-render the timed views, no grad)
    stats = []
    with torch.no_grad():
        for v in sorted(set(views_used))[:16]:
            s = _settings(cams[v], gauss, bg)
            act = (gauss.get_xyz, gauss.get_opacity, gauss.get_scaling, gauss.get_rotation, gauss.get_features)
            e = torch.Tensor([])
            out = _C.rasterize_gaussians(s.bg, act[0], e, act[1], act[2], act[3], 1.0, e, s.viewmatrix,
                                         s.projmatrix, s.tanfovx, s.tanfovy, H, W, act[4], D, s.campos, False, False,
                                         0.3)
            stats.append(_C.frame_stats(out[4], out[6], Pn, W, H))
    mean_stats = {k: float(np.mean([s[k] for s in stats])) for k in stats[0]}
    # the timed loop's per-Gaussian backward also preprocesses the next step's frame (rr_next_frame)
    mean_stats["next_frame"] = bool(trainer.fused and trainer.fuse_next and not trainer.sharded)
    # the same frame statistics at the c2f stress dilation (first timed view)
    c2f_stats = {}
    with torch.no_grad():
        s = _settings(cams[views_used[0]], gauss, bg)
        act = (gauss.get_xyz, gauss.get_opacity, gauss.get_scaling, gauss.get_rotation, gauss.get_features)
        e = torch.Tensor([])
        for lp in (30.0, 300.0):
            out = _C.rasterize_gaussians(s.bg, act[0], e, act[1], act[2], act[3], 1.0, e, s.viewmatrix,
                                         s.projmatrix, s.tanfovx, s.tanfovy, H, W, act[4], D, s.campos, False, False,
                                         lp)
            c2f_stats[str(lp)] = {k: int(v) for k, v in _C.frame_stats(out[4], out[6], Pn, W, H).items()}

    roofline = None
    kernels = {}
    for name, (ms, cnt) in breakdown.items():
        if cnt:
            # per step (= per frame): early-stop binning runs the binning stages in two phases
            kernels[name] = {"ms_per_step": ms / PW, "launches_per_step": cnt / PW, "total_ms": ms}
    sharded = getattr(trainer, "_owner", None) is not None
    if dom_timed and dom_timed[1]:
        # per frame; the sharded step's owner kernel may run as several row-chunk launches
        byts = algorithmic_bytes(dom, mean_stats, Pn, W, H, (D + 1) ** 2, world, sharded)
        launches_per_step = max(1, round(dom_timed[1] / K))
        byts = byts / launches_per_step
        dom_ms = dom_timed[0] / dom_timed[1]  # HIP events around every launch inside the timed loop
        gbs = byts / (dom_ms * 1e-3) / 1e9
        rmw_gbs = _rmw_peak(dev)
        roofline = {"kernel": dom, "step_dominant": step_dom, "bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "measured_copy_GBps": _copy_peak(dev),
                    # gauss_bwd's bytes are mostly the fused Adam's in-place read-modify-write of
                    # (param, exp_avg, exp_avg_sq): priced against that pattern measured alone
                    "measured_rmw_GBps": rmw_gbs,
                    "frac_of_measured_rmw": round(gbs / rmw_gbs, 4),
                    "ms_per_launch": round(dom_ms, 5), "launches": int(dom_timed[1]),
                    "frac": round(gbs / HBM_PEAK_GBS, 4),
                    # PMC passes are committed for the headline workload only (tools/pmc_workload.py)
                    "traffic": _pmc_traffic(dom) if (P, W, H) == (1_000_000, 1920, 1080) else None,
                    "algorithmic_bytes_per_launch": int(byts),
                    "launches_per_step": launches_per_step,
                    # the blend kernels are VALU-issue bound, not HBM bound: fraction of SIMD
                    # cycles issuing a VALU op, from the committed SQ counter pass
                    "valu_busy": _pmc_field(dom, "valu_busy") if (P, W, H) == (1_000_000, 1920, 1080) else None,
                    # VALU issue roofline from the SQ_INSTS_VALU pass: wave instructions x 2 cycles
                    # over (duration x 1024 SIMDs x 2.4 GHz) -- the bound the blend kernels sit on
                    "valu_issue_frac": (_pmc_field(dom, "valu_issue_frac")
                                        if (P, W, H) == (1_000_000, 1920, 1080) else None)}
        for k in kernels:
            b = algorithmic_bytes(k, mean_stats, Pn, W, H, (D + 1) ** 2, world, sharded)
            if b is not None:
                kernels[k]["algorithmic_GBps"] = round(b / (kernels[k]["ms_per_step"] * 1e-3) / 1e9, 1)
        # north_star states its roofline target on the per-tile blend: both blends' HBM fractions
        # (event-timed in the profiled window) and VALU-issue fractions (committed SQ pass)
        headline = (P, W, H) == (1_000_000, 1920, 1080)
        for k in ("blend_fwd", "blend_bwd"):
            if k in kernels and "algorithmic_GBps" in kernels[k]:
                roofline[k] = {"ms_per_step": round(kernels[k]["ms_per_step"], 5),
                               "achieved_GBps": kernels[k]["algorithmic_GBps"],
                               "frac": round(kernels[k]["algorithmic_GBps"] / HBM_PEAK_GBS, 4),
                               "traffic": _pmc_traffic(k) if headline else None,
                               "valu_issue_frac": _pmc_field(k, "valu_issue_frac") if headline else None}

    # the CPU baseline on every line (north_star: iters/s at 1, 2, 4, 8 GPUs "alongside the CPU
    # baseline"): rank 0 times the oracle on the same frame; the other ranks wait at the barrier
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = _cpu_baseline(gauss, cams[views_used[0]], bg, D, args.cpu_threads)
        if world > 1:
            cpu["note"] = (f"rank 0 of {world}, timed after the GPU legs while the other ranks idle; the "
                           f"oracle renders one view per iteration, so it is the same figure at every N")
    if world > 1:
        dist.barrier()

    line = {
        "metric": "train iters/sec + forward Mpix/sec, 1M Gaussians @ 1080p, 1/2/4/8 MI355X",
        "value": round(iters_per_s, 3),
        # the reference loop's densify/prune share (1 iteration in 100) priced in: the measured window
        # when it holds one, else the ordinary steps plus 1/100 of the measured extra cost of a
        # densify iteration (densify_iter_ms - ordinary_iter_ms_alone)
        "iters_per_s_1in100": round(world * 1000.0 / ms_1in100, 3),
        "unit": "train iters/s",
        "n_gpus": world,
        "steps": K,
        "warmup": Wm,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (seeded random Gaussians, 200 Fibonacci-sphere cameras, GT = render of a second random model)",
        "config": {"workload": f"train.py iteration (render fwd + L1/SSIM + bwd + densify stats + "
                               f"densify/prune every 100 it + Adam), {P} Gaussians, {W}x{H}, SH {D}, "
                               f"view-sharded dp{world}",
                   "gaussians": P, "width": W, "height": H, "sh_degree": D, "views": args.views,
                   "parallelism": (f"dp{world} (view-parallel, Gaussian-sharded: RCCL all-to-all of per-view "
                                   f"records)" if world > 1 else "dp1 (RCCL exchange forced)" if force else "dp1"),
                   "iterations": [start_iter, end_iter], "densify_events_in_window": n_densify},
        # the timed step plus the reference's per-iteration `loss.item()` host read-back (train.py:120)
        "sync_loss_iters_per_s": round(world * 1000.0 / sync_ms, 3),
        "sync_loss_ms_per_step": round(sync_ms, 4),
        "sync_loss_window": [sync_it0 + 3, sync_end],
        "densify_iter_ms": round(one_ms[D1], 3),
        "ordinary_iter_ms_alone": round(one_ms[D1 - 1], 3),
        "densify_extra_ms": round(densify_extra_ms, 3),
        "forward_mpix_per_s": round(fwd_mpix, 2),
        "forward_outputs": "color+depth+normal" if args.aux_normal else "color+depth",
        "views_per_s": round(iters_per_s, 3),  # one view per rank per step: = value
        "bracket_iters_per_s": round(world * 1000.0 / bracket_ms, 3),
        "bracket_ms": round(bracket_ms, 4),
        "c2f_low_pass_bracket_ms": c2f_ms,
        # num_rendered: the reference's bounding-square pair count; num_pairs: pairs after exact
        # culling; num_binned: pairs the early-stop binning actually sorted and blended
        "c2f_low_pass_frame_stats": c2f_stats,
        "api_iters_per_s": round(world * 1000.0 / api_ms, 3),
        "api_ms_per_step": round(api_ms, 4),
        "api_path": "unchanged train.py loop over this package's modules: render() -> GaussianRasterizer (autograd) "
                    "-> GaussianModel getters (autograd) -> HIP L1+SSIM (autograd) -> the optimizer "
                    "GaussianModel.training_setup builds (FusedAdam: torch.optim.Adam's state and arithmetic, one "
                    "launch); no densify event in the window",
        # the same loop with the stock torch.optim.Adam swapped in (foreach on ROCm: ~1.5 ms of
        # device time per step at 59M parameters, profiles/r03_api_step_trace.txt)
        "api_torch_adam_iters_per_s": round(world * 1000.0 / api_ta_ms, 3),
        "gaussians_after": int(Pn),
        "frame_stats": {k: int(v) for k, v in mean_stats.items()},
        "roofline": roofline,
        "kernels": kernels,
        "kernels_window": f"{PW} untimed profiled iterations between warmup and the timed loop (all stages event-timed)",
        "cpu_baseline": cpu,
    }
    if rank == 0:
        os.write(out_fd, (json.dumps(line) + "\n").encode())
    if world > 1 or force:
        dist.destroy_process_group()


def _clear_window(start, n):
    """First iteration s >= start such that s .. s+n-1 holds no densify / reset iteration (no
    multiple of 100: train.py:136-143)."""
    s = start
    while any(i % 100 == 0 for i in range(s, s + n)):
        s = (s // 100 + 1) * 100 + 1
    return s


def _timed_steps(trainer, it0, n, world, dev, sync_loss=False):
    """ms per training step over iterations it0+3 .. it0+2+n (three untimed first), max over ranks."""
    import torch
    import torch.distributed as dist

    for it in range(it0, it0 + 3):
        trainer.step(it, sync_loss=sync_loss)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for it in range(it0 + 3, it0 + 3 + n):
        info = trainer.step(it, sync_loss=sync_loss)
        assert not sync_loss or info.loss is not None
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        t = float(e.item())
    return 1000.0 * t / n


def _bracket(trainer, cams, gts, n, world, dev, low_pass=None):
    """ms per render-forward + loss + backward (the reference's iter_start..iter_end bracket,
    train.py:71-117), max over ranks.  Gradients go to the parameters' .grad buffers; no Adam.
    low_pass: the 2-D dilation to render with (default: the trainer's current one)."""
    import torch
    import torch.distributed as dist

    from rain_amd import fused
    from rain_amd.loss import l1_ssim_backward, l1_ssim_forward

    g, lam = trainer.g, trainer.opt.lambda_dssim
    g.bind_flat_grad(extra=0, zero=False)
    cache = fused.BinningCache()
    grads = None

    def one(i):
        nonlocal grads
        cam = cams[i % len(cams)]
        lp = trainer.low_pass if low_pass is None else low_pass
        image, _r, _d, st = fused.forward(g, cam, trainer.background, lp, cache=cache)
        loss, _p, lws = l1_ssim_forward(image, gts[i % len(cams)], lam)
        dimg = l1_ssim_backward(image, gts[i % len(cams)], lam, lws)
        grads = dict(xyz=g._xyz.grad, f_dc=g._features_dc.grad, f_rest=g._features_rest.grad,
                     opacity=g._opacity.grad, scaling=g._scaling.grad, rotation=g._rotation.grad)
        fused.backward(st, dimg, grads, None, None)

    with torch.no_grad():
        for i in range(3):
            one(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(n):
            one(i)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
    g.optimizer.zero_grad(set_to_none=True)
    if world > 1:
        e = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        t = float(e.item())
    return 1000.0 * t / n


def _api_leg(gauss, cams, gts, opt, pipe, extent, it0, n, world, dev, torch_adam=True):
    """ms per train iteration on the reference-API path (Trainer(fused=False)): render() ->
    GaussianRasterizer autograd -> getters autograd -> fused L1+SSIM -> Adam.  torch_adam: the stock
    torch.optim.Adam the reference's gaussian_model.py builds (gaussian_model.py:153, foreach on
    ROCm), else this package's GaussianModel default, FusedAdam (one launch for all groups); state
    carried over from the fused run.  Iterations it0.. (it0 = 1 + a multiple of 100: no densify /
    reset inside)."""
    import torch
    import torch.distributed as dist

    from rain_amd.train import TrainConfig, Trainer

    fused_opt = gauss.optimizer
    if torch_adam:
        groups = [{"params": g["params"], "lr": g["lr"], "name": g["name"]} for g in fused_opt.param_groups]
        adam = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        for g in fused_opt.param_groups:
            p = g["params"][0]
            if p in fused_opt.state and len(fused_opt.state[p]):
                st = fused_opt.state[p]
                adam.state[p] = {"step": st["step"].detach().clone().cpu().float().reshape(()),
                                 "exp_avg": st["exp_avg"].detach().clone(),
                                 "exp_avg_sq": st["exp_avg_sq"].detach().clone()}
        gauss.optimizer = adam
    tr = Trainer(gauss, cams, gts, opt, pipe, TrainConfig(seed=1), scene_extent=extent, fused=False)
    it = it0
    for _ in range(3):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(n):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    gauss.optimizer = fused_opt
    if world > 1:
        e = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        t = float(e.item())
    return 1000.0 * t / n


def _copy_peak(dev):
    """Achievable HBM rate: read + write bytes / time of the library's float4 streaming copy
    (rt_stream_copy, the MI355X guide's ~6.3 TB/s yardstick), 1 GiB buffers, HIP events on the
    stream the copy is launched on."""
    import torch

    from rain_amd import _native

    L = _native.train_lib()
    a = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    st = _native.stream_of(a)

    def copy():
        if L.rt_stream_copy(b.data_ptr(), a.data_ptr(), a.numel() * 4, st) != 0:
            raise RuntimeError(L.rt_last_error().decode())

    for _ in range(3):
        copy()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        copy()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    del a, b
    return round(2 * (1 << 30) / (ms * 1e-3) / 1e9, 1)


def _rmw_peak(dev):
    """Achievable rate of Adam's in-place access pattern: read + write bytes / time of the
    library's three-array read-modify-write stream (rt_stream_rmw: param, exp_avg, exp_avg_sq of
    59M floats, the bench model's parameter count), HIP events on its stream.  The fused-Adam
    backward moves mostly these bytes; on MI355X this pattern runs well below a copy."""
    import torch

    from rain_amd import _native

    L = _native.train_lib()
    n = 59_000_000
    buf = torch.zeros(3 * n, dtype=torch.float32, device=dev)
    p, m, v = buf[:n], buf[n:2 * n], buf[2 * n:]
    st = _native.stream_of(buf)

    def rmw():
        if L.rt_stream_rmw(p.data_ptr(), m.data_ptr(), v.data_ptr(), n, st) != 0:
            raise RuntimeError(L.rt_last_error().decode())

    for _ in range(3):
        rmw()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        rmw()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    del buf
    return round(6 * 4 * n / (ms * 1e-3) / 1e9, 1)


def _host_cpus():
    """(threads the CPU baseline may use, description of the host): every CPU this process is
    allowed to run on, capped by a cgroup CPU quota when one is set (the GPU box gives each GPU a
    16-CPU share of a larger machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    use = min(aff, quota) if quota else aff
    return use, {"host_cpu_count": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                 "cpu_model": model}


def _settings(cam, gauss, bg):
    from rain_amd.synthetic import settings_for

    return settings_for(cam, gauss.active_sh_degree, bg=bg)


def _pmc_field(kernel, field):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get("kernels", {}).get(kernel, {}).get(field)
    except (OSError, ValueError):
        return None


def _pmc_traffic(kernel):
    """HBM bytes per launch from a committed rocprofv3 PMC pass (tools/pmc_traffic.py), else null."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        v = d.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")
        return int(v) if v is not None else None
    except (OSError, ValueError):
        return None


def _cpu_baseline(gauss, cam, bg, D, threads, views=3):
    """The oracle (test infrastructure, `port` of the reference algorithm) on the same frame."""
    import numpy as np
    import torch

    from oracle import oracle as O

    O.build()
    avail, host = _host_cpus()
    nthr = threads or avail
    with torch.no_grad():
        s = _settings(cam, gauss, bg)
        m = gauss.get_xyz.detach().float().cpu().numpy()
        op = gauss.get_opacity.detach().float().cpu().numpy()
        sc = gauss.get_scaling.detach().float().cpu().numpy()
        ro = gauss.get_rotation.detach().float().cpu().numpy()
        sh = gauss.get_features.detach().float().cpu().numpy()
    st = O.Settings(image_height=s.image_height, image_width=s.image_width, tanfovx=s.tanfovx, tanfovy=s.tanfovy,
                    bg=s.bg.cpu().numpy(), scale_modifier=1.0, viewmatrix=s.viewmatrix.cpu().numpy(),
                    projmatrix=s.projmatrix.cpu().numpy(), sh_degree=D, campos=s.campos.cpu().numpy(),
                    low_pass=0.3)
    dpix = np.random.default_rng(0).standard_normal((3, s.image_height, s.image_width)).astype(np.float32)
    tf = tb = 0.0
    for _ in range(views):  # the same frame `views` times: a bounded sample of ~10 s
        t0 = time.perf_counter()
        nr, color, radii, depth, state = O.forward(st, m, op, shs=sh, scales=sc, rotations=ro, nthreads=nthr)
        t1 = time.perf_counter()
        O.backward(state, st, m, radii, dpix, shs=sh, scales=sc, rotations=ro, nthreads=nthr)
        t2 = time.perf_counter()
        tf += t1 - t0
        tb += t2 - t1
    return {"value": round(views / (tf + tb), 4), "unit": "render fwd+bwd iters/s", "cores": int(O.lib().orc_threads()),
            "kind": "port",
            "sample": f"{views} x 1 full {s.image_width}x{s.image_height} view, {m.shape[0]} Gaussians, SH {D}: forward "
                      f"{tf / views:.2f}s + backward {tb / views:.2f}s per view (rasterizer only; loss/Adam not included)",
            "forward_mpix_per_s": round(views * s.image_width * s.image_height / tf / 1e6, 4), **host}


if __name__ == "__main__":
    sys.exit(main())
