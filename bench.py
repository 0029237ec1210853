#!/usr/bin/env python3
"""bench.py -- Mrays/s of the MI355X volume ray-marcher on BASELINE.json's metric configuration.

Workload (BASELINE.json `metric`, SURVEY.md 8d "north-star metric config"): V_shell(1024) fp32
volume (synthetic, generated in HBM), 1920x1080 image, Henyey-Greenstein shading with the two
lights of examples/example1.m:36, on-the-fly gradient, Fe=1 Fr=0.4 Fa=0.6, color [1 1 0],
threshold 0.9, camera rotate(125,25,0), f=3, dist=6, reflection = the class default Volume(1).

A "step" = one frame: the ray-march kernel over this rank's image columns (+ at N>1 the RCCL
gather of the column partitions to rank 0 and the on-device assembly of the full image).
Volumes are resident in HBM before the timed region (sync_volumes is not timed).  The K timed
frames run one after the other on one HIP stream -- what a synchronous VolumeRender.render user
gets per frame (minus the D2H copy) -- so `value` / `ms_per_step` are the serial frame rate and
`ms_per_step` >= the march kernel's own time.  A second, separately reported pass
(`pipelined`, --pipelined-streams, default 2) issues independent frames of a movie round-robin on
several streams so that one frame's tail overlaps the next frame's start; it is not `value`.
Run: python bench.py [--gpus N --steps K --warmup W]; N>1 under torch.distributed.run.
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

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD at 2.4 GHz
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles")
VALU_ISSUE_PER_S = 1024 * 2.4e9 / 2
METRIC = "Mrays/s + achieved HBM GB/s, 1024³ vol @ 1920×1080 HG-shaded, 1/2/4/8 GPU"


def workload_name(n, W, H, L, gradient):
    """config.workload; also the key profiles/<round>/traffic.json must carry for roofline.traffic."""
    return (f"V_shell({n}) fp32 {n}^3, {W}x{H}, "
            + ("HG 2 lights (example1.m), on-the-fly gradient" if (L == 2 and gradient == "compute")
               else f"HG {L} lights, {gradient} gradient (diagnostic)")
            + ", rotate(125,25,0) f=3 dist=6 thr=0.9")


def launched_lanes(timed_kernels):
    """Depth lanes K of the march kernel the timed frames launched (its first template argument)."""
    if not timed_kernels:
        return None
    name = max(timed_kernels, key=timed_kernels.get)
    head = name.split("march_kernel<", 1)
    return int(head[1].split(",", 1)[0]) if len(head) == 2 else None


def rotation(alpha, beta, gamma):
    """VolumeRender.rotate from identity (exact cosd/sind at multiples of 90)."""
    from volume_renderer_amd.volume_render import _cosd, _sind
    ca, sa, cb, sb, cg, sg = _cosd(alpha), _sind(alpha), _cosd(beta), _sind(beta), _cosd(gamma), _sind(gamma)
    rx = np.array([[1, 0, 0], [0, ca, -sa], [0, sa, ca]])
    ry = np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
    rz = np.array([[cg, -sg, 0], [sg, cg, 0], [0, 0, 1]])
    return np.eye(3) @ rx @ ry @ rz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--volume", type=int, default=1024, help="V_shell edge (metric config: 1024); not --n, which torch.distributed.run would take for its own --nnodes")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--block-cols", type=int, default=16, help="column block of the image partition")
    ap.add_argument("--cpu-stride", type=int, default=8, help="CPU baseline: every k-th column")
    ap.add_argument("--cpu-stride-1core", type=int, default=96, help="1-core CPU baseline: every k-th column")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: every CPU this process may use -- affinity and cgroup quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gradient", choices=["compute", "lookup"], default="compute",
                    help="lookup: precomputed gradient volumes (example1_grad.m, BASELINE config 3), made on "
                         "the device with vr_gradient_device")
    ap.add_argument("--lights", type=int, default=2, help="light sources (0: emission-absorption only; "
                    "diagnostics, the metric config has 2)")
    ap.add_argument("--rotate", type=float, nargs=3, default=[125.0, 25.0, 0.0],
                    help="camera rotate(alpha, beta, gamma) (metric config: 125 25 0; others are diagnostics)")
    ap.add_argument("--sim-parts", type=int, default=0,
                    help="diagnostic (1 GPU): also time each rank's share of a P-way column partition, "
                         "the kernel time a rank would see at --gpus P")
    ap.add_argument("--pipelined-streams", type=int, default=2,
                    help="extra pass (not `value`): the frames issued round-robin on this many HIP streams "
                         "(independent frames of a movie, example3.m); 1 or 0 skips it")
    ap.add_argument("--movie", type=int, default=30,
                    help="frames of each movie pass (0: none; world size 1): frame i seen from rotate(start) * "
                         "rotate(step)^i, as examples/example2.m:53-66 turns the camera before every render -- no "
                         "frame has an earlier frame of its camera; reported apart from `value`")
    ap.add_argument("--movie-step", type=float, nargs=3, default=[0.0, 12.0, 0.0],
                    help="camera turn between movie frames, rotate(alpha, beta, gamma) (example2.m: 0 12 0)")
    ap.add_argument("--movie-starts", default="125,25,0;30,10,0",
                    help="';'-separated start cameras of the movie passes, rotate(alpha,beta,gamma) from identity")
    ap.add_argument("--chunk-stats-k", action="store_true",
                    help="diagnostic (a VR_COUNT_K=1 build): also the chunk statistics of the production "
                         "depth lanes (the default counted launch runs at K = 1)")
    ap.add_argument("--gather", choices=["overlap", "serial"], default="overlap",
                    help="N > 1: frame i's gather to rank 0 overlapped with frame i + 1's render (two part "
                         "buffers, parallel.FrameGather), or finished before the next frame starts")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (RCCL over xGMI, the product); gloo: a rehearsal of the N > 1 path with every "
                         "rank on the visible GPUs round-robin (several on one GPU), collectives on host copies")
    ap.add_argument("--traffic-json", default=_latest_traffic_json(),
                    help="PMC-measured HBM bytes per launch of the march kernel (tools/profile_summary.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        if world == 1 and args.gpus > 1:
            sys.exit("bench.py --gpus N>1 must be launched with torch.distributed.run --nproc-per-node N")
    gloo = args.dist_backend == "gloo"
    if gloo:  # rehearsal: ranks dealt round-robin to the visible GPUs (device_count does not initialise HIP)
        local_rank %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import volume_renderer_amd as vr
    from volume_renderer_amd import mex
    if os.environ.get("VR_TEST_SWITCHES") == "1" or args.chunk_stats_k:
        # A/B runs (tools/gpupass.py) select kernel variants through VR_* switches, which the library
        # reads only with its test switches on (include/vrhip.h vr_set_option)
        mex.enable_test_switches()

    dev = torch.device("cuda", local_rank)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    n, W, H = args.volume, args.width, args.height

    # ---- inputs, resident in HBM before timing ------------------------------------------------
    # the volume is made on rank 0 only (what one H2D upload of the MATLAB array gives) and, at N > 1,
    # broadcast once to every rank's replica over RCCL, timed apart from the frames
    vol_t = torch.empty(n * n * n, dtype=torch.float32, device=dev)
    if rank == 0:
        mex.synth_shell_device(vol_t.data_ptr(), n, sptr)
    torch.cuda.synchronize(dev)
    from volume_renderer_amd import parallel
    if world > 1 and gloo:  # (gloo: through a host copy)
        vol_h = vol_t.cpu()
        bcast = parallel.broadcast_volume(vol_h, world, rank)
        vol_t.copy_(vol_h)
        del vol_h
    else:
        bcast = parallel.broadcast_volume(vol_t, world, rank) if world > 1 else None
    em = mex.DeviceVolume(vol_t.data_ptr(), (n, n, n), last_update=10, owner=vol_t)
    refl = vr.Volume(1)          # VolumeRender.m:131 default VolumeReflection
    refl.TimeLastUpdate = np.uint64(5)
    lut = vr.Volume(vr.HenyeyGreenstein(64))
    lut.TimeLastUpdate = np.uint64(7)
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]
    lights = (lights * ((args.lights + 1) // 2))[: args.lights]
    h = vr.volumeRender("new")
    grads = []
    if args.gradient == "lookup":  # Volume.grad on the device, 4 arrays resident
        grads = [torch.empty_like(vol_t) for _ in range(3)]
        mex.gradient_device(vol_t.data_ptr(), (n, n, n), *[g.data_ptr() for g in grads], sptr)
        torch.cuda.synchronize(dev)
        gvols = [mex.DeviceVolume(g.data_ptr(), (n, n, n), last_update=11 + i, owner=g) for i, g in enumerate(grads)]
        vr.volumeRender("sync_volumes", h, np.uint64(0), em, refl, em, *gvols)
    else:
        vr.volumeRender("sync_volumes", h, np.uint64(0), em, refl, em)  # Em, Re, Ab (Ab aliases Em)
    R = rotation(*args.rotate)
    ra, keep = mex.render_args(lights, lut, np.float32([1.0, 0.4, 0.6]), np.float32([1, 1, 1]),
                               np.uint64([H, W]), np.flip(R, 0).astype(np.float32), np.float32([0, 3.0, 6.0]),
                               np.float32(0.9), np.float32([1, 1, 0]))
    host_vol = vol_t.cpu().numpy() if (rank == 0 and world == 1 and not args.no_cpu_baseline) else None
    del vol_t, grads  # the library holds its own resident copies

    part = mex.partition(args.block_cols, rank, world) if world > 1 else None
    my_cols = mex.partition_columns(W, part)
    max_cols = max(mex.partition_columns(W, mex.partition(args.block_cols, p, world)) for p in range(world)) \
        if world > 1 else W
    full = torch.zeros(3 * W * H, dtype=torch.float32, device=dev) if rank == 0 else None
    # N > 1: the per-frame gather of the parts to rank 0 and the assembly there (parallel.FrameGather:
    # two part buffers, frame i's gather overlapped with frame i + 1's render unless --gather serial)
    fg = None
    if world > 1:
        def assemble(gath, _i):
            mex.assemble_partitions(gath.data_ptr(), W, H, args.block_cols, world, max_cols, full.data_ptr(), sptr)
        fg = parallel.FrameGather(3 * max_cols * H, world, rank, device=dev, staged=gloo, assemble=assemble)
        out_local = fg.buffer(0)
    else:
        out_local = torch.zeros(3 * max_cols * H, dtype=torch.float32, device=dev)
    steps_t = torch.zeros(48, dtype=torch.int64, device=dev)

    # sample count of this rank's launch (exact, counter variant; untimed)
    mex.render_device(h, ra, out_local.data_ptr(), part, steps_t.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    my_samples = int(steps_t[0].item())
    my_lit = int(steps_t[1].item())
    chunk_stats = [int(v) for v in steps_t[2:5].tolist()]
    wave_stats = [int(v) for v in steps_t[5:7].tolist()]
    fail_hist = [int(v) for v in steps_t[8:40].tolist()]
    staged_by_s = [int(v) for v in steps_t[40:44].tolist()]
    probe_stats = [int(steps_t[7].item()), int(steps_t[44].item())]
    prod_stats = None
    if args.chunk_stats_k:  # the same counted launch at the production K (vr_capi.hip VR_COUNT_PROD)
        steps_t.zero_()
        os.environ["VR_COUNT_PROD"] = "1"
        try:
            mex.render_device(h, ra, out_local.data_ptr(), part, steps_t.data_ptr(), sptr)
            torch.cuda.synchronize(dev)
        finally:
            del os.environ["VR_COUNT_PROD"]
        kn = mex.last_march_kernel() or ""
        if "march_kernel<1," in kn:  # a normal build counts at K = 1 only (VR_COUNT_PROD needs VR_COUNT_K=1)
            print("bench.py: --chunk-stats-k needs a VR_COUNT_K=1 build; the counted launch ran at K = 1",
                  file=sys.stderr)
        prod_stats = {"kernel": kn,
                      "chunks_staged_leaped_global": [int(v) for v in steps_t[2:5].tolist()],
                      "wave_iterations_total_lit": [int(v) for v in steps_t[5:7].tolist()],
                      "staged_chunks_by_S_32_16_8_4": [int(v) for v in steps_t[40:44].tolist()],
                      "global_chunk_box_hist_256": [int(v) for v in steps_t[8:40].tolist()]}

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    timed_kernels = {}  # march kernel instantiation -> timed frames that launched it
    nframe = [0]  # frames rendered so far (the part buffer alternates with it at N > 1)

    def frame(i=None):
        k = nframe[0]
        nframe[0] += 1
        buf = fg.buffer(k) if fg is not None else out_local
        if i is not None:
            ev[i][0].record(stream)
        mex.render_device(h, ra, buf.data_ptr(), part, 0, sptr)
        if i is not None:
            ev[i][1].record(stream)
            kn = mex.last_march_kernel()
            timed_kernels[kn] = timed_kernels.get(kn, 0) + 1
        if fg is not None:
            fg.start(k)  # issues this frame's gather, finishes (and on rank 0 assembles) the previous one
            if args.gather == "serial":
                fg.flush()

    for _ in range(args.warmup):
        frame()
    if fg is not None:
        fg.flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        frame(i)
    if fg is not None:
        fg.flush()  # the last frame's gather and assembly, inside the timed region
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    t_kernel_s = sum(kern_ms) / len(kern_ms) / 1e3
    cdev = torch.device("cpu") if gloo else dev  # device of the small report tensors
    ranks = None
    if world > 1:  # per-rank kernel time and the per-frame time beyond it (the exposed gather +
        # assembly, waiting for the slowest rank included), all-gathered to rank 0
        exposed = max(0.0, elapsed / args.steps * 1e3 - t_kernel_s * 1e3)
        ranks = parallel.rank_report(t_kernel_s * 1e3, exposed, world, rank, device=cdev)
        if ranks is not None:
            ranks["gather"] = args.gather
            ranks["what"] = ("mean over the timed frames: march kernel (HIP events around each rank's launch); "
                             "gather_assembly = the rank's time per frame beyond its kernel (the exposed part of "
                             "the gather to rank 0 and, on rank 0, of the assembly; waiting for the slowest rank "
                             "included)")

    # ---- extra pass (not `value`): independent frames round-robin on several streams ----------
    pipe_elapsed = None
    ns = args.pipelined_streams if not (world > 1 and gloo) else 0  # (the rehearsal skips this pass)
    if ns > 1:
        streams = [torch.cuda.Stream(dev) for _ in range(ns)]
        outs = [torch.zeros_like(out_local) for _ in range(ns)]
        fulls = [torch.zeros(3 * W * H, dtype=torch.float32, device=dev) for _ in range(ns)] if rank == 0 else None
        gaths = ([torch.zeros_like(fg.gath[0]) for _ in range(ns)] if (world > 1 and rank == 0) else None)

        def oframe(i):
            j = i % ns
            mex.render_device(h, ra, outs[j].data_ptr(), part, 0, streams[j].cuda_stream)
            if world > 1:  # gather + assembly on the default stream, after this frame's kernel only
                stream.wait_stream(streams[j])
                dist.gather(outs[j], list(gaths[j].chunk(world)) if rank == 0 else None, dst=0)
                if rank == 0:
                    mex.assemble_partitions(gaths[j].data_ptr(), W, H, args.block_cols, world, max_cols,
                                            fulls[j].data_ptr(), sptr)
                streams[j].wait_stream(stream)  # the buffers of frame i are reused by frame i + ns

        for i in range(max(args.warmup, 2 * ns)):  # every stream's schedule measured (vr_capi.hip)
            oframe(i)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for i in range(args.steps):
            oframe(i)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        pipe_elapsed = time.perf_counter() - t1
        del outs, fulls, gaths

    sim = None
    if args.sim_parts > 1 and world == 1:
        P_ = args.sim_parts
        pcols = max(mex.partition_columns(W, mex.partition(args.block_cols, p, P_)) for p in range(P_))
        sim_out = torch.zeros(3 * pcols * H, dtype=torch.float32, device=dev)
        sim = []
        for p in range(P_):
            pp = mex.partition(args.block_cols, p, P_)
            mex.render_device(h, ra, sim_out.data_ptr(), pp, 0, sptr)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(3):
                mex.render_device(h, ra, sim_out.data_ptr(), pp, 0, sptr)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            sim.append(round(e0.elapsed_time(e1) / 3, 3))
        del sim_out

    movies = None
    if args.movie > 0 and world == 1:
        movies = movie_passes(args, mex, h, lights, lut, W, H, stream, sptr, dev, out_local.numel())

    samples_all = torch.tensor([my_samples, my_lit], dtype=torch.int64, device=cdev)
    el = torch.tensor([elapsed, pipe_elapsed or 0.0], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(samples_all, op=dist.ReduceOp.SUM)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed, pipe_elapsed = float(el[0].item()), (float(el[1].item()) if pipe_elapsed is not None else None)
    total_samples = int(samples_all[0].item())
    total_lit = int(samples_all[1].item())

    result = None
    if rank == 0:
        rays = W * H
        ms_per_step = elapsed / args.steps * 1e3
        value = rays * args.steps / elapsed / 1e6
        L, G = args.lights, (6 if args.gradient == "compute" else 3)
        F = 1 + ((G + 1 + L) if L > 0 else 0)  # trilinear fetches per sample, SURVEY.md 8d
        bytes_launch = 4.0 * my_samples * F + 12.0 * my_cols * H
        achieved = bytes_launch / t_kernel_s / 1e9
        # the fetches a sample really needs: every sample its centre fetch, only the shaded ones the
        # F - 1 gradient / reflection / LUT fetches (opacity-0 samples add exactly 0)
        fetched = 4.0 * (my_samples + my_lit * (F - 1)) + 12.0 * my_cols * H
        result = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic V_shell(%d) (SURVEY.md 8d), generated in HBM" % n,
            "config": {"workload": workload_name(n, W, H, L, args.gradient)
                       + ("" if list(args.rotate) == [125.0, 25.0, 0.0]
                          else " [diagnostic camera rotate(%g,%g,%g)]" % tuple(args.rotate)),
                       "volume": [n, n, n], "image": [W, H], "lights": L, "gradient": args.gradient,
                       "parallelism": f"image-column partition x{world} (block {args.block_cols})"
                       + (" + RCCL gather" if world > 1 else ""),
                       "depth_lanes": launched_lanes(timed_kernels)
                       or mex.depth_lanes(my_cols, H, 6.0 * n / (W * 3.0)),  # dist * n / (W * f)
                       "frames": "serial, one HIP stream" + (
                           "; the gather of frame i overlapped with the render of frame i + 1"
                           if world > 1 and args.gather == "overlap" else "")},
            "samples_per_frame": total_samples,
            "shaded_samples_per_frame": total_lit,
            "chunks_staged_leaped_global": chunk_stats,
            "wave_iterations_total_lit": wave_stats,
            "global_chunk_box_hist_256": fail_hist,
            "staged_chunks_by_S_32_16_8_4": staged_by_s,
            "probe_runs_leaped_failed": probe_stats,
            "gb_per_s_sample_stream": round(4.0 * total_samples * F / (elapsed / args.steps) / 1e9, 1),
            # achieved / frac: the bytes the samples need (SURVEY 8d's "minimum fetches needed to
            # reproduce the output" once opacity-0 samples are elided exactly: their shading adds exactly
            # 0) per launch over the march kernel's mean HIP-event time
            "roofline": {"bound": "hbm", "achieved": round(fetched / t_kernel_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(fetched / t_kernel_s / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": None,
                         "kernel_ms": round(t_kernel_s * 1e3, 3),
                         "kernel": max(timed_kernels, key=timed_kernels.get) if timed_kernels else None,
                         "kernels_timed": timed_kernels,
                         "bytes_per_launch": fetched,
                         "algorithmic_bytes": "4 B x (samples + shaded samples x (F-1)) + 12 B x pixels, F = %d "
                                              "(every sample its centre fetch; the shaded ones, opacity > 0, also "
                                              "the gradient / reflection / LUT fetches)" % F,
                         "sample_stream": {"bytes_per_launch": bytes_launch, "achieved": round(achieved, 1),
                                           "frac": round(achieved / HBM_PEAK_GBS, 4),
                                           "what": "SURVEY 8d's definitional 4 B x samples x F + 12 B x pixels: "
                                                   "every sample charged F fetches, opacity-0 ones (60.5 % at the "
                                                   "metric config, leaped or unshaded) included, so it can exceed "
                                                   "1"},
                         "sample_stream_frac": round(achieved / HBM_PEAK_GBS, 4),
                         "valu": None},
            "cpu_baseline": None,
        }
        if pipe_elapsed is not None:
            result["pipelined"] = {"streams": ns, "ms_per_step": round(pipe_elapsed / args.steps * 1e3, 3),
                                   "mrays_s": round(rays * args.steps / pipe_elapsed / 1e6, 3),
                                   "what": "the same frames issued round-robin on several HIP streams "
                                           "(independent movie frames overlap their tails); not `value`"}
        if ranks is not None:
            result["ranks"] = ranks
        if bcast is not None:
            result["upload_broadcast_ms"] = bcast["ms"]
            result["volume_broadcast"] = bcast
        if prod_stats is not None:
            result["chunk_stats_production_k"] = prod_stats
        if movies is not None:
            for m in movies:
                m["median_over_fixed_kernel"] = round(m["median_ms"] / (t_kernel_s * 1e3), 3)
            result["movie"] = movies
        if sim is not None:
            result["sim_parts_kernel_ms"] = {"parts": args.sim_parts, "per_part": sim, "max": max(sim),
                                             "est_speedup": round(t_kernel_s * 1e3 / max(sim), 2)}

    if rank == 0:  # the frame's identity, also without the CPU baseline (A/B runs); at N > 1 the last
        # frame assembled from the gathered parts -- the same bytes as the one-GPU frame
        import hashlib
        img = out_local if world == 1 else full
        result["image_sha256"] = hashlib.sha256(
            np.ascontiguousarray(img[: 3 * W * H].view(3, W, H).cpu().numpy()).tobytes()).hexdigest()

    # ---- CPU baseline: the oracle's sources at -O3 (C, OpenMP) on a column sample of the frame -----
    if rank == 0 and world == 1 and host_vol is not None:
        result["cpu_baseline"], result["parity_sampled_columns"] = cpu_baseline(
            args, host_vol, n, W, H, refl, lut, lights, R, full if world > 1 else out_local)

    if rank == 0:
        # roofline.traffic / .valu: per-launch HBM bytes and VALU instructions of the march kernel
        # from the rocprofv3 PMC passes committed under profiles/ (tools/profile_summary.py;
        # FETCH_SIZE x 2 KiB + WRITE_SIZE KiB, the x2 being the gfx950 64-B-per-128-B-request tally);
        # only when they were measured on this workload.
        try:
            with open(args.traffic_json) as fh:
                tj_all = json.load(fh)
            # one entry per measured workload (round 4: every BASELINE config), or a round-3 file
            cands = tj_all.get("entries", [tj_all])
            tj = next((e for e in cands if e.get("workload") == result["config"]["workload"]
                       and e.get("kernel") == result["roofline"]["kernel"]), {})
            if world == 1 and tj:
                src = os.path.relpath(args.traffic_json, ROOT)
                result["roofline"]["traffic"] = tj["bytes_per_launch"]
                result["roofline"]["traffic_source"] = src + " (" + tj.get("method", "") + ")"
                vi = tj.get("valu_insts_per_launch")
                if vi:
                    peak = VALU_ISSUE_PER_S
                    result["roofline"]["valu"] = {
                        "insts_per_launch": vi, "achieved": round(vi / t_kernel_s / 1e9, 2),
                        "peak": round(peak / 1e9, 1), "unit": "G wave64-instr/s",
                        "frac": round(vi / t_kernel_s / peak, 4),
                        "source": src + " (SQ_INSTS_VALU; peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 "
                                        "VALU instruction, MI355X_MICROARCH.md)"}
        except (OSError, ValueError, KeyError):
            pass
        result["roofline"]["binding"] = binding_roof(result["roofline"], t_kernel_s)
        print(json.dumps(result), flush=True)
    vr.volumeRender("delete", h)
    if world > 1:
        dist.destroy_process_group()


def movie_passes(args, mex, h, lights, lut, W, H, stream, sptr, dev, out_floats):
    """Movies (examples/example2.m:53-66): from each start camera, args.movie frames, each turned by
    args.movie_step from the previous one, rendered back to back on the bench's stream with HIP events
    around each frame.  Every frame is a camera the library has not rendered before (the first frame
    of the metric start aside, which the fixed-camera frames rendered), so its block schedule comes
    from the occupancy-map prediction, not from a measurement (vr_capi.hip attach_schedule)."""
    import hashlib
    step = rotation(*args.movie_step)
    out = []
    for spec in args.movie_starts.split(";"):
        start = [float(v) for v in spec.split(",")]
        R = rotation(*start)
        ras, keep, bufs = [], [], []
        for _ in range(args.movie):
            ra, kp = mex.render_args(lights, lut, np.float32([1.0, 0.4, 0.6]), np.float32([1, 1, 1]),
                                     np.uint64([H, W]), np.flip(R, 0).astype(np.float32),
                                     np.float32([0, 3.0, 6.0]), np.float32(0.9), np.float32([1, 1, 0]))
            ras.append(ra)
            keep.append(kp)
            bufs.append(torch.empty(out_floats, dtype=torch.float32, device=dev))
            R = R @ step
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in ras]
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for (e0, e1), ra, b in zip(evs, ras, bufs):
            e0.record(stream)
            mex.render_device(h, ra, b.data_ptr(), None, 0, sptr)
            e1.record(stream)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        ms = [a.elapsed_time(b) for a, b in evs]
        dig = hashlib.sha256()
        for b in bufs:
            dig.update(np.ascontiguousarray(b[: 3 * W * H].cpu().numpy()).tobytes())
        med = float(np.median(ms))
        out.append({"start": start, "step": list(args.movie_step), "frames": len(ms),
                    "frame_ms": [round(v, 3) for v in ms], "median_ms": round(med, 3), "max_ms": round(max(ms), 3),
                    "first_ms": round(ms[0], 3), "max_over_median": round(max(ms) / med, 3),
                    "wall_ms_per_frame": round(wall / len(ms) * 1e3, 3), "frames_sha256": dig.hexdigest(),
                    "what": "frame i at rotate(start) * rotate(step)^i, HIP events around each render; no frame "
                            "repeats a camera (frame 0 of the metric start is the fixed-camera frame)"})
        del bufs
    return out


def binding_roof(rf, t_kernel_s):
    """The roof nearest to binding the launch: the largest of the fractions that describe hardware
    use -- the bytes the samples need (`frac`, "fetched"), the HBM bytes the counters saw (FETCH_SIZE x
    2 + WRITE_SIZE, over 8 TB/s) and the VALU issue rate (over its wave64 peak).  The F-weighted sample
    stream (`sample_stream_frac`) is a definitional figure (it charges F fetches to opacity-0 samples,
    which the kernel skips; it reads above 1), so it is not a candidate."""
    cands = {"fetched": rf["frac"]}
    if rf.get("traffic"):
        cands["hbm_traffic"] = round(rf["traffic"] / t_kernel_s / 1e9 / HBM_PEAK_GBS, 4)
    if rf.get("valu"):
        cands["valu"] = rf["valu"]["frac"]
    name = max(cands, key=cands.get)
    return {"roof": name, "frac": cands[name], "candidates": cands,
            "note": "max of the hardware-use fractions; none near 1 means the launch is latency-bound "
                    "(waits the resident waves do not hide), DESIGN.md s5"}


def cpu_share():
    """CPUs this process may use: its affinity mask, capped by a cgroup-v2 CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline_lib():
    """The CPU baseline's library: the oracle's sources rebuilt here with -O3 -march=native when gcc
    is present (a few seconds), else the prebuilt -O3 -march=x86-64-v3 oracle/libcpubase.so."""
    import subprocess
    import tempfile
    od = os.path.join(ROOT, "oracle")
    out = os.path.join(tempfile.mkdtemp(prefix="vr_cpubase_"), "libcpubase_native.so")
    flags = ["-O3", "-march=native", "-fPIC", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-fopenmp"]
    try:
        subprocess.run(["gcc", *flags, "-shared", "-o", out, os.path.join(od, "vr_oracle.c"),
                        os.path.join(od, "vr_oracle_host.c"), "-lm"], check=True, capture_output=True, timeout=120)
        return out, "gcc " + " ".join(flags)
    except (OSError, subprocess.SubprocessError):
        return os.path.join(od, "libcpubase.so"), "prebuilt oracle/libcpubase.so (-O3 -march=x86-64-v3)"


def cpu_baseline(args, host_vol, n, W, H, refl, lut, lights, R, gpu_out):
    """The oracle's scalar C restatement at -O3, OpenMP over columns, on every CPU this process may
    use and on one core, each on a column sample of the same frame; plus the sampled-column diff
    of the GPU image against it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    path, build = cpu_baseline_lib()
    share = cpu_share()
    threads = args.cpu_threads or share
    S = O.OracleSession()
    oh = S.new()
    ovol = O.OVolume(host_vol.reshape((n, n, n), order="F"), 10)
    S.sync_volumes(oh, 0, ovol, O.OVolume(refl.Data, 5), ovol)
    L6 = np.array([list(l.Position) + list(l.Color) for l in lights], np.float32)
    rargs = (L6, O.OVolume(lut.Data, 7), [1.0, 0.4, 0.6], [1, 1, 1], [H, W], np.flip(R, 0).astype(np.float32),
             [0, 3.0, 6.0], 0.9, [1, 1, 0])

    def run(stride, nthreads):
        cols = np.arange(0, W, stride, dtype=np.int64)
        t1 = time.perf_counter()
        img, samples = S.render(oh, *rargs, threads=nthreads, cols=cols, lib_path=path)
        return cols, img, samples, time.perf_counter() - t1

    cols, img, cpu_samples, cpu_s = run(args.cpu_stride, threads)
    cols1, _, samples1, cpu1_s = run(args.cpu_stride_1core, 1)
    g = gpu_out[: 3 * W * H].view(3, W, H).cpu().numpy()
    o = np.transpose(img, (2, 1, 0))  # [H,W,3] F-order -> (3, W, H) C-order view
    d = np.abs(g[:, cols, :] - o[:, cols, :])
    base = {
        "value": round(len(cols) * H / cpu_s / 1e6, 5), "unit": "Mrays/s", "cores": threads,
        "kind": "port",
        "sample": f"oracle/vr_oracle.c (scalar C restatement, OpenMP over columns; {build}) on every "
                  f"{args.cpu_stride}th column ({len(cols)} cols x {H} rays, {cpu_samples} samples) of the same "
                  f"frame, {cpu_s:.1f} s on {threads} threads",
        "host_cpus": os.cpu_count(), "cpu_share": share,
        "one_core": {"value": round(len(cols1) * H / cpu1_s / 1e6, 6), "unit": "Mrays/s", "cores": 1,
                     "sample": f"every {args.cpu_stride_1core}th column ({len(cols1)} cols x {H} rays, "
                               f"{samples1} samples), {cpu1_s:.1f} s"}}
    import hashlib
    c, xi, y = np.unravel_index(int(np.argmax(d)), d.shape)
    x = int(cols[xi])
    parity = {"max_abs": float(d.max()), "img_max": float(np.abs(o[:, cols, :]).max()),
              "bit_exact_frac": float((g[:, cols, :].view(np.uint32) == o[:, cols, :].view(np.uint32)).mean()),
              "max_abs_at": {"x": x, "y": int(y), "channel": "RGB"[int(c)], "product": float(g[c, x, y]),
                             "oracle": float(o[c, x, y])},
              "image_sha256": hashlib.sha256(np.ascontiguousarray(g).tobytes()).hexdigest(),
              "what": "GPU frame vs the oracle (fp32) on every %dth column; image_sha256 = the whole GPU frame's "
                      "[3][W][H] fp32 bytes" % args.cpu_stride}
    return base, parity


def _latest_traffic_json():
    """profiles/<latest round>/traffic.json (the newest PMC pass committed)."""
    import glob
    c = sorted(glob.glob(os.path.join(ROOT, "profiles", "round*", "traffic.json")),
               key=lambda p: int("".join(ch for ch in os.path.basename(os.path.dirname(p)) if ch.isdigit()) or 0))
    return c[-1] if c else os.path.join(ROOT, "profiles", "round1", "traffic.json")


if __name__ == "__main__":
    main()
