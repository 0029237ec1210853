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
