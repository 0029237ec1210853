"""Sort-last slab protocol on CPU: world_size 2 and 3 over gloo.

A stand-in for vr_render_slab with the same contract (per-ray state: premultiplied colour, alpha,
"goes on", and the resume point -- here the index of the ray's next sample; a slab composites
only the samples it owns, in ray order, stops a ray at sum.a > thr, and hands it off at its first
sample beyond the slab; direction 0 marches both kinds of ray) checks the pipelined two-sweep
hand-off of volume_renderer_amd.parallel: the result must equal compositing every ray's samples
in one process, bit for bit, and no slab may replay a sample before it (every ray resumes where
the previous slab stopped).  The kernel itself is checked
against the one-volume render on the GPU (test_gpu_parity.py::test_sort_last_slabs_...)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from volume_renderer_amd import parallel

NRAY, NSAMP, DEPTH, NTILES, THR = 50, 40, 30.0, 4, 0.9


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rays():
    """Per ray: sample z positions (monotone along the ray, either direction) and (c, a) values."""
    rng = np.random.default_rng(7)
    z0 = rng.uniform(0, DEPTH, NRAY).astype(np.float32)
    dz = rng.uniform(-1.5, 1.5, NRAY).astype(np.float32)
    z = z0[:, None] + dz[:, None] * np.arange(NSAMP, dtype=np.float32)[None, :]
    c = rng.uniform(0, 1, (NRAY, NSAMP)).astype(np.float32)
    a = (rng.uniform(0, 1, (NRAY, NSAMP)) ** 4).astype(np.float32) * 0.3
    return z, dz, c, a


def _composite(state, c, a):
    om = np.float32(1) - state[1]
    state[0] = np.float32(om * c * a + state[0])
    state[1] = np.float32(om * a + state[1])
    return state[1] > THR


def _reference():
    z, dz, c, a = _rays()
    out = np.zeros((NRAY, 2), np.float32)
    for i in range(NRAY):
        s = np.zeros(2, np.float32)
        for k in range(NSAMP):
            if _composite(s, c[i, k], a[i, k]):
                break
        out[i] = s
    return out


def _tile_rays(t):
    return np.arange(t, NRAY, NTILES)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z, dz, c, a = _rays()
        z0, z1 = parallel.slab_bounds(int(DEPTH), world)[rank]

        replayed = [0]

        def render_tile(t, direction, fresh, buf):  # stand-in for vr_render_slab on tile t
            st = buf.numpy().reshape(4, -1)            # planes: colour, alpha, goes-on, resume index
            for j, i in enumerate(_tile_rays(t)):
                if direction != 0 and (dz[i] >= 0) != (direction > 0):
                    if fresh:
                        st[:, j] = (0, 0, 1, 0)
                    continue
                s = np.zeros(2, np.float32) if fresh else st[:2, j].copy()
                go = True if fresh else st[2, j] != 0
                k = 0 if fresh else int(st[3, j])      # resume at the next sample
                past = False
                while go and k < NSAMP:
                    zk = z[i, k]
                    if not (z0 <= zk < z1):
                        if (zk >= z1) if dz[i] >= 0 else (zk < z0):
                            past = True
                            break
                        replayed[0] += 1               # before the slab
                        k += 1
                        continue
                    stop = _composite(s, c[i, k], a[i, k])
                    k += 1
                    if stop:
                        break
                st[:2, j] = s
                st[2, j] = 1.0 if past else 0.0
                st[3, j] = k

        states = [torch.zeros(4 * len(_tile_rays(t))) for t in range(NTILES)]
        parallel.sort_last_sweeps(render_tile, states, world, rank)
        if rank == 0:
            out = np.zeros((NRAY, 2), np.float32)
            for t in range(NTILES):
                st = states[t].numpy().reshape(4, -1)
                out[_tile_rays(t)] = st[:2].T
                assert not st[2].any()
            q.put((out, replayed[0]))
        else:
            assert replayed[0] == 0
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_pipelined_slab_sweeps_equal_one_volume(world):
    """world 1: one process renders each tile once (direction 0, both kinds of ray)."""
    ref = _reference()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, replayed = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert replayed == 0  # every slab resumed at the ray's next sample: nothing replayed


def test_slab_bounds_partition_the_depth():
    b = parallel.slab_bounds(100, 4)
    assert b[0][0] == -float("inf") and b[-1][1] == float("inf")
    assert all(b[i][1] == b[i + 1][0] for i in range(3)) and b[1] == (25.0, 50.0)
