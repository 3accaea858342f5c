"""Row partition + strip gather for N GPUs, one process per GPU.

The reference renders on 16 std::threads over contiguous pixel batches
(rt_in_one_weekend/main.cpp:318-338) and has no multi-GPU path.  Here row j
goes to rank j % N (interleaved: per-row cost is uneven, contiguous strips
would cap 8-GPU scaling at 6.08x vs 7.86x); each rank renders its
rows into a strip of ceil(H/N) rows with rt_render_rows; ONE gather over
torch.distributed (backend "nccl" = RCCL over xGMI on the GPU box, "gloo" in
the CPU tests) brings the strips to rank 0, which un-permutes them.  Every
pixel's RNG stream is keyed by its image coordinates, so the image is
bit-identical for any N.
"""
import numpy as np


def strip_rows(H, rank, world):
    """(row0, row_step, nrows): rank's rows are row0 + k*row_step, k < nrows.
    nrows is the same on every rank (ceil(H/N)); rows >= H are zero-filled."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return rank, world, (H + world - 1) // world


def gather_strips(strip, rank, world, dst=0, async_op=False, group=None):
    """Gather every rank's strip tensor to `dst` (one collective).  Returns the
    list of strips on dst, None elsewhere; with async_op, (that list, the
    collective's Work): the strips are valid, and `strip` may be overwritten,
    only after Work.wait() (for RCCL that makes the caller's current stream
    wait for the collective, without blocking the host).  `group`: a process
    group over all ranks (rank numbers as in the default group), or None."""
    import torch.distributed as dist

    if world == 1 and not (dist.is_available() and dist.is_initialized()):  # no process group: nothing to gather
        return ([strip], None) if async_op else [strip]
    bufs = [strip.new_empty(strip.shape) for _ in range(world)] if rank == dst else None
    work = dist.gather(strip, gather_list=bufs, dst=dst, async_op=async_op, group=group)
    return (bufs, work) if async_op else bufs


def unpermute(strips, H):
    """Interleaved strips (rank g holds rows g, g+N, ...) -> image [H, W, 3]."""
    world = len(strips)
    nrows, W, C = strips[0].shape
    out = np.zeros((H, W, C), dtype=np.asarray(strips[0]).dtype)
    for g, s in enumerate(strips):
        s = np.asarray(s)
        rows = np.arange(g, H, world)
        out[rows] = s[: len(rows)]
    return out
