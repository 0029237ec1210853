"""Image-space partition across GPUs: one process per GPU, each holding a replica
of the volume, renders an interleaved set of column blocks; rank 0 gathers the parts over RCCL
(xGMI) and assembles the full image on the device (vr_assemble_partitions).

Columns are cut into blocks of `block_cols`; block b belongs to part b % num_parts (interleaving
balances the strongly position-dependent ray cost).  A part's buffer is the column-major
[H, cols, 3] image of its columns in increasing x, padded to the largest part so the gather has
equal-sized messages.  This module is backend-agnostic (RCCL on the GPU, gloo in CPU tests).
"""
from __future__ import annotations

import numpy as np


def partition_column_indices(width: int, block_cols: int, part: int, num_parts: int) -> np.ndarray:
    """Global x of every column part `part` owns, in its buffer order (matches the kernel's
    local-column -> x mapping in vr_kernels.hip and vr_partition_columns)."""
    nblocks = (width + block_cols - 1) // block_cols
    cols = [b * block_cols + i for b in range(part, nblocks, num_parts) for i in range(block_cols)
            if b * block_cols + i < width]
    return np.asarray(cols, dtype=np.int64)


def partition_layout(width: int, block_cols: int, num_parts: int):
    """(columns per part, max columns) of the partition."""
    counts = [len(partition_column_indices(width, block_cols, p, num_parts)) for p in range(num_parts)]
    return counts, max(counts) if counts else 0


def gather_partitions(local, gathered, world: int, rank: int, group=None) -> None:
    """Gather every rank's (equal-sized, padded) part buffer into `gathered` on rank 0.
    `gathered` is a flat tensor of world * local.numel() on rank 0 (ignored elsewhere)."""
    import torch.distributed as dist
    if world == 1:
        if rank == 0 and gathered is not None and gathered.data_ptr() != local.data_ptr():
            gathered.copy_(local)
        return
    dist.gather(local, list(gathered.chunk(world)) if rank == 0 else None, dst=0, group=group)


class FrameGather:
    """The per-frame gather of the column parts to rank 0, overlapped with the next frame's render
    (bench.py at N > 1): two part buffers per rank (and two gather buffers on rank 0) alternate
    between frames, so frame i's gather runs on the collective's own stream while frame i + 1
    renders.  Usage per frame i: render into `buffer(i)` (enqueued on the current stream), then
    `start(i)`; after the last frame `flush()`.  `start(i)` issues frame i's gather (asynchronous;
    it waits for the render on the device) and finishes frame i - 1's: the current stream waits for
    that gather (RCCL; gloo: the host waits), then rank 0 runs `assemble(gathered, frame)` on it.
    A buffer is written again two frames later, after its gather has been waited for.

    staged=True: for a backend without device-tensor collectives (gloo driving GPU buffers in a
    rehearsal on one GPU), each part goes through a host copy.  Backend-agnostic otherwise (RCCL on
    the GPU, gloo on CPU tensors in the test)."""

    def __init__(self, part_numel: int, world: int, rank: int, device=None, dtype=None, staged: bool = False,
                 assemble=None, group=None):
        import torch
        dtype = dtype or torch.float32
        self.world, self.rank, self.group, self.staged, self.assemble = world, rank, group, staged, assemble
        self.bufs = [torch.zeros(part_numel, dtype=dtype, device=device) for _ in range(2)]
        self.gath = ([torch.zeros(world * part_numel, dtype=dtype, device=device) for _ in range(2)]
                     if rank == 0 else None)
        if staged:
            self.hbufs = [torch.zeros(part_numel, dtype=dtype) for _ in range(2)]
            self.hgath = [torch.zeros(world * part_numel, dtype=dtype) for _ in range(2)] if rank == 0 else None
        self.pending = None

    def buffer(self, i: int):
        return self.bufs[i % 2]

    def start(self, i: int) -> None:
        import torch.distributed as dist
        slot = i % 2
        if self.staged:
            self.hbufs[slot].copy_(self.bufs[slot])  # (synchronous: after the render)
            src, dst = self.hbufs[slot], self.hgath[slot] if self.rank == 0 else None
        else:
            src, dst = self.bufs[slot], self.gath[slot] if self.rank == 0 else None
        work = dist.gather(src, list(dst.chunk(self.world)) if self.rank == 0 else None, dst=0, group=self.group,
                           async_op=True)
        prev, self.pending = self.pending, (work, slot, i)
        if prev is not None:
            self._finish(*prev)

    def _finish(self, work, slot: int, i: int) -> None:
        work.wait()
        if self.rank == 0:
            if self.staged:
                self.gath[slot].copy_(self.hgath[slot])
            if self.assemble is not None:
                self.assemble(self.gath[slot], i)

    def flush(self) -> None:
        if self.pending is not None:
            prev, self.pending = self.pending, None
            self._finish(*prev)


def volume_checksum(vol):
    """An order-sensitive checksum of a volume's bytes (int64, device-side for a GPU tensor): the sum of
    its 32-bit words weighted by their index mod 65521, plus their plain sum -- equal on two replicas
    iff (with overwhelming probability) their bytes are."""
    import torch
    flat = vol.reshape(-1).view(torch.int32)
    acc = torch.zeros(2, dtype=torch.int64, device=flat.device)
    step = 1 << 26  # chunks: the int64 temporaries stay at 1.5 GiB whatever the volume
    for i0 in range(0, flat.numel(), step):
        w = flat[i0:i0 + step].to(torch.int64)
        idx = torch.arange(i0, i0 + w.numel(), device=w.device, dtype=torch.int64) % 65521 + 1
        acc[0] += (w * idx).sum()
        acc[1] += w.sum()
    return acc


def broadcast_volume(vol, world: int, rank: int, src: int = 0, group=None) -> dict:
    """The one-time volume distribution of SURVEY.md 8e ("Collectives"): the volume, resident on rank
    `src` (uploaded or generated there), broadcast in place into every rank's replica buffer (RCCL
    over xGMI on the GPU; gloo in the CPU test).  Timed with the backend's own completion (device
    synchronise around it on a GPU), reported apart from the per-frame time; each replica's checksum
    is all-gathered so that rank 0 can state that every rank holds the same bytes."""
    import time

    import torch
    import torch.distributed as dist
    nbytes = vol.numel() * vol.element_size()
    if world == 1:
        return {"bytes": int(nbytes), "ms": 0.0, "gb_per_s": None, "ranks": 1, "replicas_identical": True}
    cuda = vol.is_cuda
    if cuda:
        torch.cuda.synchronize(vol.device)
    dist.barrier(group=group)
    t0 = time.perf_counter()
    dist.broadcast(vol, src=src, group=group)
    if cuda:
        torch.cuda.synchronize(vol.device)
    dist.barrier(group=group)
    ms = (time.perf_counter() - t0) * 1e3
    mine = volume_checksum(vol)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    same = all(bool(torch.equal(a, allv[src])) for a in allv)
    t = torch.tensor([ms], dtype=torch.float64, device=vol.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    ms = float(t.item())
    return {"bytes": int(nbytes), "ms": round(ms, 3), "gb_per_s": round(nbytes / ms / 1e6, 2) if ms > 0 else None,
            "ranks": world, "replicas_identical": same, "backend": str(dist.get_backend(group)),
            "what": "one-time dist.broadcast of the volume from rank %d (barrier to barrier, max over ranks); "
                    "not part of the per-frame time" % src}


def rank_report(kernel_ms: float, gather_ms: float, world: int, rank: int, device=None, group=None):
    """Per-rank attribution of a multi-GPU frame (bench.py at N > 1): every rank's mean march-kernel
    time (HIP events around its launch) and its gather + assembly time (from the end of its launch
    to the end of the RCCL gather -- on rank 0 also the on-device assembly; it includes waiting for
    the slowest rank's kernel), all-gathered; and how many ranks the collective saw (an all-reduce of
    ones).  Returns the dict on rank 0, None elsewhere.  Backend-agnostic (RCCL on the GPU, gloo in
    the CPU test)."""
    import torch
    import torch.distributed as dist
    mine = torch.tensor([float(kernel_ms), float(gather_ms)], dtype=torch.float64, device=device)
    if world > 1:
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine, group=group)
        one = torch.ones(1, dtype=torch.int64, device=device)
        dist.all_reduce(one, group=group)
        seen, backend = int(one.item()), str(dist.get_backend(group))
    else:
        allv, seen, backend = [mine], 1, "none"
    if rank != 0:
        return None
    k = [round(float(v[0].item()), 3) for v in allv]
    g = [round(float(v[1].item()), 3) for v in allv]
    return {"ranks_seen": seen, "backend": backend,
            "kernel_ms_per_rank": k, "kernel_ms_max": max(k), "kernel_ms_min": min(k),
            "kernel_imbalance": round(max(k) / min(k), 4) if min(k) > 0 else None,
            "gather_assembly_ms_per_rank": g, "gather_assembly_ms_rank0": g[0],
            "what": "mean over the timed frames: march kernel (HIP events around each rank's launch); "
                    "gather + assembly = end of the rank's launch to the end of the gather (rank 0: + "
                    "the on-device assembly; includes waiting for the slowest rank)"}


# ---- sort-last z-slabs -----------------------------------------
# Volumes larger than one GPU: rank r holds only the planes of z-slab r (vr_slab_planes) and
# marches only the samples that slab owns (vr_render_slab).  A ray's samples are composited in ray
# order by handing the exact ray state (premultiplied rgb, alpha, "goes on", and the resume point:
# t, position and sample index of its next sample) from slab to slab: rays with dir.z >= 0 visit
# the slabs in ascending z (rank 0 -> world-1), the others descending (world-1 -> 0), each slab
# continuing the march where the previous one stopped.  The descending rays start in the top slab,
# so the last rank marches both kinds in one launch (direction 0) and the descending sweep proper
# runs over ranks world-2 .. 0.  The image is cut into `ntiles` column tiles (vr_partition parts)
# so that the ranks work on different tiles at the same time: rank r renders tile t of the
# ascending sweep once rank r-1 has sent it, then the descending sweep runs back down; rank 0 ends
# with every ray's final state, bit-identical to the one-volume render.

def slab_bounds(depth: int, world: int):
    """Owned ranges [z0, z1) of `world` equal z-slabs of a depth-`depth` volume (the end slabs
    open towards -inf / +inf so that no sample is left without an owner)."""
    cuts = [round(depth * r / world) for r in range(1, world)]
    return [(-float("inf") if r == 0 else float(cuts[r - 1]), float("inf") if r == world - 1 else float(cuts[r]))
            for r in range(world)]


def sort_last_sweeps(render_tile, states, world: int, rank: int, group=None, streams=None) -> None:
    """Run the two pipelined sweeps.  `render_tile(t, direction, fresh, buf)` renders this rank's
    slab for tile t in place on buf (direction +1 / -1, or 0 = both on the top slab; fresh: the
    tile's rays start here, no incoming state) on the current stream; `states[t]` is this rank's
    state buffer of tile t (a tensor the backend can send).  On return rank 0's buffers hold the
    final state of every tile.  One process (world 1) renders each tile once, both directions.
    streams (optional, device tensors): tile t's receive, render and send run on streams[t % n], so
    that consecutive tiles' launches overlap their tails; the current stream waits for them all."""
    import contextlib

    import torch
    import torch.distributed as dist
    last = rank == world - 1
    on = (lambda t: torch.cuda.stream(streams[t % len(streams)])) if streams else (lambda t: contextlib.nullcontext())
    if streams:
        for s in streams:  # the buffers and the volume were produced on the current stream
            s.wait_stream(torch.cuda.current_stream())
    pending = []
    # ascending sweep: rank 0 starts every tile fresh; the top slab also starts the descending rays
    for t, buf in enumerate(states):
        with on(t):
            if rank > 0:
                dist.recv(buf, src=rank - 1, group=group)
            render_tile(t, 0 if last else +1, rank == 0, buf)
            if not last:
                pending.append(dist.isend(buf, dst=rank + 1, group=group))
    for w in pending:
        w.wait()
    pending = []
    # descending sweep: the top slab hands its tiles down (sent only now, so that every pair of
    # ranks sees its messages in one order: the ascending ones first)
    for t, buf in enumerate(states):
        with on(t):
            if not last:
                dist.recv(buf, src=rank + 1, group=group)
                render_tile(t, -1, False, buf)
            if rank > 0:
                pending.append(dist.isend(buf, dst=rank - 1, group=group))
    for w in pending:
        w.wait()
    if streams:
        for s in streams:
            torch.cuda.current_stream().wait_stream(s)
