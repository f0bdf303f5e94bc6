"""Frame-batch data parallelism across the GPUs of one node.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on
the box, "gloo" in the CPU tests).  Frames shard as contiguous ranges, each
rank runs the whole detect+describe path on its own frames (no halo, no
data-path collective), and the only exchange is ONE all-gather of the
compacted result slabs (layout: include/surfhip.h, surfhip_pack_slab) so
every rank ends up holding every frame's keypoints and descriptors.

torch is passed in by the caller; this module never imports it (a GPU
process must load torch before libsurfhip so that one HIP runtime serves
both).
"""
from __future__ import annotations

import numpy as np


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous shard of rank r: frames [r*n/R, (r+1)*n/R) -> (start, count)."""
    start = (rank * n_total) // world
    stop = ((rank + 1) * n_total) // world
    return start, stop - start


def agree_slab_size(dist, torch, used: int, device) -> int:
    """All ranks agree on the collective size: the max used slab bytes."""
    t = torch.tensor([int(used)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def allgather_slabs(dist, torch, slab, cap: int, world: int, out=None, async_op: bool = False):
    """All-gather `cap` bytes of every rank's slab into out[world * cap]
    (uint8).  Returns (out, work-or-None)."""
    src = slab[:cap]
    if out is None:
        out = torch.empty(world * cap, dtype=torch.uint8, device=src.device)
    dst = out[:world * cap]
    if dist.get_backend() == "gloo":
        chunks = list(dst.view(world, cap).unbind(0))
        work = dist.all_gather(chunks, src, async_op=async_op)
    else:
        work = dist.all_gather_into_tensor(dst, src, async_op=async_op)
    return out, work


def split_gathered(gathered: np.ndarray, world: int, cap: int, parse):
    """Per-rank (counts, points, desc) from the gathered byte buffer."""
    g = np.ascontiguousarray(gathered[:world * cap]).reshape(world, cap)
    return [parse(g[r]) for r in range(world)]
