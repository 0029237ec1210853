"""Multi-process partition protocol on CPU: world_size 2 over gloo.

Each rank renders its interleaved column blocks (here with the CPU oracle standing in for the
GPU kernel: the test is about the partition, the padded part layout and the gather, which are
backend-agnostic), packs them into the part buffer layout of vr_render_device
(c*max_cols*H + j*H + y), rank 0 gathers the parts with volume_renderer_amd.parallel and scatters
them into the full image; the result must equal the single-process render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from volume_renderer_amd import parallel

W, H, BLOCK = 37, 29, 4


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    vol = O.OVolume(O.shell_volume(24), 10)
    lut = O.OVolume(O.hg_lut(16, 0.8), 7)
    lights = np.array([[500, 1000, 550, 0, 1, 1], [0, 550, 90, 1, 0.5, 1]], np.float32)
    R = O.rotation(125, 25, 0)
    return vol, lut, lights, R


def _render(cols=None):
    vol, lut, lights, R = _scene()
    S = O.OracleSession()
    h = S.new()
    S.sync_volumes(h, 0, vol, O.OVolume(np.ones((1, 1, 1), np.float32), 5), vol)
    img, _ = S.render(h, lights, lut, [1.0, 0.4, 0.6], [1, 1, 1], [H, W], np.flip(R, 0).astype(np.float32),
                      [0, 3.0, 6.0], 0.9, [1, 1, 0], threads=1, cols=cols)
    S.delete(h)
    return img  # [H, W, 3]


def _assemble(parts: np.ndarray, world: int, max_cols: int) -> np.ndarray:
    """Host restatement of vr_assemble_partitions: part p's local column j -> global x."""
    full = np.zeros((H, W, 3), np.float32)
    for p in range(world):
        idx = parallel.partition_column_indices(W, BLOCK, p, world)
        slab = parts[p].reshape(3, max_cols, H)
        for j, x in enumerate(idx):
            full[:, x, :] = slab[:, j, :].T
    return full


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        counts, max_cols = parallel.partition_layout(W, BLOCK, world)
        idx = parallel.partition_column_indices(W, BLOCK, rank, world)
        img = _render(cols=idx)
        buf = np.zeros((3, max_cols, H), np.float32)
        buf[:, : len(idx), :] = np.transpose(img[:, idx, :], (2, 1, 0))
        local = torch.from_numpy(buf.reshape(-1))
        gathered = torch.zeros(world * local.numel()) if rank == 0 else None
        parallel.gather_partitions(local, gathered, world, rank)
        if rank == 0:
            q.put(_assemble(gathered.numpy().reshape(world, -1), world, max_cols))
    finally:
        dist.destroy_process_group()


def _report_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r reports kernel 10 + r ms, gather 1 + 0.5 r ms
        rep = parallel.rank_report(10.0 + rank, 1.0 + 0.5 * rank, world, rank)
        if rank == 0:
            q.put(rep)
        else:
            assert rep is None
    finally:
        dist.destroy_process_group()


def _bcast_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 0 holds the volume (V_shell), the others an empty replica buffer of the same size
        vol = torch.from_numpy(np.ascontiguousarray(O.shell_volume(40).reshape(-1, order="F")))
        if rank != 0:
            vol = torch.full_like(vol, -1.0)
        rep = parallel.broadcast_volume(vol, world, rank)
        q.put((rank, vol.numpy().copy(), rep))
    finally:
        dist.destroy_process_group()


def test_volume_broadcast_replicates_rank0_bytes():
    """bench.py at N > 1 (SURVEY.md 8e "Collectives"): the volume is made on rank 0 only and broadcast
    once (parallel.broadcast_volume, RCCL on the GPU, gloo here at world 2); every rank then holds rank
    0's bytes exactly, and the report carries the bytes, the time and the replicas' checksum check."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (v, rep)) for r, v, rep in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = np.ascontiguousarray(O.shell_volume(40).reshape(-1, order="F"))
    for r in range(world):
        v, rep = got[r]
        assert np.array_equal(v.view(np.uint32), ref.view(np.uint32)), r
        assert rep["bytes"] == ref.nbytes and rep["ranks"] == world and rep["replicas_identical"] is True
        assert rep["ms"] >= 0 and rep["backend"] == "gloo"
    # a replica that differs is caught by the checksum (order-sensitive)
    a = torch.from_numpy(ref.copy())
    b = a.clone()
    i, j = int(np.argmax(ref)), int(np.argmin(ref))
    assert ref[i] != ref[j]
    b[[i, j]] = b[[j, i]]
    assert torch.equal(parallel.volume_checksum(a), parallel.volume_checksum(a.clone()))
    assert not torch.equal(parallel.volume_checksum(a), parallel.volume_checksum(b))


def test_rank_report_attributes_a_multi_gpu_frame():
    """bench.py's per-rank report at N > 1 (parallel.rank_report), over gloo at world 2: every rank's
    kernel and gather + assembly times reach rank 0 in rank order, with their max / min and the
    number of ranks the collective saw."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_report_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    rep = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert rep["ranks_seen"] == 2 and rep["backend"] == "gloo"
    assert rep["kernel_ms_per_rank"] == [10.0, 11.0] and rep["kernel_ms_max"] == 11.0 and rep["kernel_ms_min"] == 10.0
    assert rep["gather_assembly_ms_per_rank"] == [1.0, 1.5] and rep["gather_assembly_ms_rank0"] == 1.0
    assert rep["kernel_imbalance"] == 1.1


@pytest.mark.parametrize("world", [2])
def test_partitioned_render_gathers_to_the_full_image(world):
    ref = _render()
    assert ref.max() > 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_partition_layout_covers_every_column_once():
    for world in (1, 2, 3, 8):
        counts, max_cols = parallel.partition_layout(W, BLOCK, world)
        allc = np.sort(np.concatenate([parallel.partition_column_indices(W, BLOCK, p, world) for p in range(world)]))
        assert np.array_equal(allc, np.arange(W)) and sum(counts) == W and max_cols == counts[0]


def _frame_gather_worker(rank, world, port, q, staged):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, frames = 257, 7
        seen = []
        fg = parallel.FrameGather(n, world, rank, staged=staged,
                                  assemble=lambda g, i: seen.append((i, g.clone().numpy())))
        for i in range(frames):
            buf = fg.buffer(i)
            # frame i's "render": a value per (frame, rank, element), written over the buffer of frame i - 2
            buf.copy_(torch.arange(n, dtype=torch.float32) + 1000.0 * rank + 1e5 * i)
            fg.start(i)
            if rank == 0:  # frame i - 1 is assembled once frame i's gather has been issued
                assert [f for f, _ in seen] == list(range(i))
        fg.flush()
        if rank == 0:
            q.put(seen)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("staged", [False, True])
def test_frame_gather_overlaps_and_keeps_every_frame(staged):
    """bench.py's per-frame gather at N > 1 (parallel.FrameGather), over gloo at world 2: frame i's
    gather is issued after its render and finished (assembled on rank 0) after frame i + 1's render
    was issued, through two alternating buffers -- every frame reaches rank 0 whole, in order, with
    each rank's part in rank order, although a buffer is rewritten two frames later; staged: the
    same through host copies (the one-GPU gloo rehearsal of the bench)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_frame_gather_worker, args=(r, world, port, q, staged)) for r in range(world)]
    for p in procs:
        p.start()
    seen = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [f for f, _ in seen] == list(range(7))
    n = 257
    for i, g in seen:
        want = np.concatenate([np.arange(n, dtype=np.float32) + 1000.0 * r + 1e5 * i for r in range(world)])
        assert np.array_equal(g, want), i
