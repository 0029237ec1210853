#!/usr/bin/env python3
"""Sort-last z-slab rendering across ranks (BASELINE config 5's "multi-pass
manager as brick partition + composite"), one process per GPU:

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/sort_last_bench.py

Rank r synthesizes only the planes of z-slab r of V_shell(n) that its samples need
(vr_slab_planes), and the frame is rendered by the two pipelined sweeps of
volume_renderer_amd.parallel.sort_last_sweeps over `--tiles` column tiles: the exact ray state
crosses from slab to slab, so rank 0's image equals the one-volume render bit for bit (--check
renders the whole volume on rank 0 and compares).  --backend gloo runs the hand-off through host
memory (a multi-process rehearsal on one GPU).  Prints one JSON line (diagnostic, not the driver's
bench line)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--volume", type=int, default=1024, help="V_shell edge")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tiles", type=int, default=16)
    ap.add_argument("--block-cols", type=int, default=16)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--streams", type=int, default=1, help="HIP streams the tiles rotate over")
    ap.add_argument("--slabs", type=int, default=0,
                    help="one process: the volume as this many z-slabs, each resident on the GPU, chained "
                         "slab after slab (the ranks' work of a sort-last frame, serialized; whole image)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ngpu = torch.cuda.device_count()
    torch.cuda.set_device(local % max(ngpu, 1))
    dev = torch.device("cuda", local % max(ngpu, 1))
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
    import volume_renderer_amd as vr
    from volume_renderer_amd import mex, parallel
    mex.enable_test_switches()  # (the VR_* variant switches this tool sets)
    from bench import rotation

    n, W, H = args.volume, args.width, args.height
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    es = [1.0, 1.0, 1.0]
    refl = vr.Volume(1)
    refl.TimeLastUpdate = np.uint64(5)
    lut = vr.Volume(vr.HenyeyGreenstein(64))
    lut.TimeLastUpdate = np.uint64(7)
    lights = [vr.LightSource([500, 1000, 550], [0, 1, 1]), vr.LightSource([0, 550, 90], [1, 0.5, 1])]

    def slab_handle(nslab, s):
        """Handle holding the planes z-slab s of nslab needs; (handle, slab bounds, planes, tensor)."""
        z0, z1 = parallel.slab_bounds(n, nslab)[s]
        first, count = mex.slab_planes((n, n, n), es, z0, z1)
        t = torch.empty(n * n * count, dtype=torch.float32, device=dev)
        mex.synth_shell_planes_device(t.data_ptr(), n, first, count, sptr)
        torch.cuda.synchronize(dev)
        em = mex.DeviceVolume(t.data_ptr(), (n, n, count), last_update=10 + s, owner=t)
        hh = vr.volumeRender("new")
        vr.volumeRender("sync_volumes", hh, np.uint64(0), em, refl, em)
        return hh, (z0, z1), (first, count), t, em

    nslab = args.slabs if (args.slabs > 1 and world == 1) else 0
    if nslab:
        chain = [slab_handle(nslab, s) for s in range(nslab)]
        h, (z0, z1), (first, count), slab_t, _ = chain[0]
    else:
        h, (z0, z1), (first, count), slab_t, _ = slab_handle(world, rank)
    R = rotation(125, 25, 0)
    ra, keep = mex.render_args(lights, lut, np.float32([1.0, 0.4, 0.6]), np.float32(es), np.uint64([H, W]),
                               np.flip(R, 0).astype(np.float32), np.float32([0, 3.0, 6.0]), np.float32(0.9),
                               np.float32([1, 1, 0]))
    parts = [mex.partition(args.block_cols, t, args.tiles) for t in range(args.tiles)]
    cols = [mex.partition_columns(W, p) for p in parts]
    dstate = [torch.zeros(mex.SLAB_PLANES * c * H, dtype=torch.float32, device=dev) for c in cols]
    host = args.backend != "nccl" and world > 1  # gloo: hand the state over through host memory
    states = [torch.zeros(mex.SLAB_PLANES * c * H, dtype=torch.float32) for c in cols] if host else dstate

    def render_tile(t, direction, fresh, buf):
        d = dstate[t]
        if host and not fresh:
            d.copy_(buf)
        mex.render_slab(h, ra, mex.slab(n, first, z0, z1, direction), 0 if fresh else d.data_ptr(), d.data_ptr(),
                        torch.cuda.current_stream(dev).cuda_stream, part=parts[t])
        if host:
            buf.copy_(d)  # synchronous copy to host

    streams = [torch.cuda.Stream(dev) for _ in range(args.streams)] if args.streams > 1 and not host else None

    def frame():
        if nslab:  # asc over the slabs (the top one both ways), then desc
            d = dstate[0]
            order = [(k, +1 if k < nslab - 1 else 0) for k in range(nslab)] + [(k, -1) for k in range(nslab - 2, -1, -1)]
            for i, (k, direction) in enumerate(order):
                hk, (a, b), (fk, _), _, emk = chain[k]
                # renders read the BOUND volumes (the last sync_volumes of any handle): rebind this
                # slab's planes (resident already: the sync only binds them)
                vr.volumeRender("sync_volumes", hk, np.uint64(0), emk, refl, emk)
                mex.render_slab(hk, ra, mex.slab(n, fk, a, b, direction), 0 if i == 0 else d.data_ptr(), d.data_ptr(),
                                sptr, part=parts[0])
            return
        parallel.sort_last_sweeps(render_tile, states, world, rank, streams=streams)

    for _ in range(args.warmup):
        frame()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        if args.backend == "nccl":
            el = el.to(dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    ms = float(el.item()) / args.steps * 1e3
    if rank == 0:
        out = {"metric": "sort-last z-slab frame (diagnostic)", "value": round(W * H / ms / 1e3, 3),
               "unit": "Mrays/s", "ms_per_frame": round(ms, 3), "ranks": world, "backend": args.backend,
               "volume": [n, n, n], "image": [W, H], "tiles": args.tiles, "slabs_one_process": nslab, "streams": args.streams, "block_cols": args.block_cols, "sched_env": os.environ.get("VR_SCHED"),
               "depth_lanes_env": os.environ.get("VR_DEPTH_LANES"), "slab_planes": [first, count]}
        if args.check:
            max_cols = max(cols)
            gathered = torch.zeros(args.tiles * 3 * max_cols * H, dtype=torch.float32, device=dev)
            for t in range(args.tiles):
                src = states[t].to(dev)[: 3 * cols[t] * H].view(3, cols[t], H)
                gathered.view(args.tiles, 3, max_cols, H)[t, :, : cols[t]].copy_(src)
            img = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)
            mex.assemble_partitions(gathered.data_ptr(), W, H, args.block_cols, args.tiles, max_cols, img.data_ptr(),
                                    sptr)
            full_t = torch.empty(n * n * n, dtype=torch.float32, device=dev)
            mex.synth_shell_device(full_t.data_ptr(), n, sptr)
            torch.cuda.synchronize(dev)
            h2 = vr.volumeRender("new")
            fv = mex.DeviceVolume(full_t.data_ptr(), (n, n, n), last_update=11, owner=full_t)
            vr.volumeRender("sync_volumes", h2, np.uint64(0), fv, refl, fv)
            ref = torch.zeros(3 * W * H, dtype=torch.float32, device=dev)
            mex.render_device(h2, ra, ref.data_ptr(), None, 0, sptr)
            torch.cuda.synchronize(dev)
            a, b = img.cpu().numpy(), ref.cpu().numpy()
            out["check"] = {"bit_identical": bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))),
                            "max_abs": float(np.abs(a - b).max()), "img_max": float(b.max())}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
