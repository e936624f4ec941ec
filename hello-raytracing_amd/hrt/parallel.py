"""Row-tile partition of the image across ranks and the one gather that assembles it.

SURVEY §8(e): every pixel is independent (seed = f(global x, global y, H, time)), so rank r of N renders
the interleaved rows r, r+N, r+2N, ... of the full image with global coordinates (rt_params.row0 = r,
row_step = N) — interleaving spreads the cheap sky rows evenly — and one collective gather over RCCL
(xGMI on one node) brings the row bands to the destination rank, which un-interleaves them. There is no
other data-path communication. Works with any torch.distributed backend (nccl = RCCL on GPUs, gloo on CPU
for the tests).
"""
from __future__ import annotations


def rows_of(rank: int, world: int, height: int) -> int:
    """Number of rows owned by `rank` (rows rank, rank+world, ... < height)."""
    return len(range(rank, height, world))


def assemble(parts, height: int, world: int, out=None):
    """Un-interleave: parts[k] holds rows k, k+world, ... (padded to the max row count)."""
    import torch

    if out is None:
        out = torch.empty((height,) + tuple(parts[0].shape[1:]), dtype=parts[0].dtype, device=parts[0].device)
    for k in range(world):
        out[k::world] = parts[k][: rows_of(k, world, height)]
    return out


def gather_image(part, height: int, dist, rank: int, world: int, dst: int = 0, gathered=None, out=None):
    """Collective: every rank passes its padded (ceil(H/world), W, 3) band; returns the full image on
    `dst` (None elsewhere). One dist.gather — the only collective of the path."""
    import torch

    if world == 1:
        return part[:height] if out is None else out.copy_(part[:height])
    if dist.get_backend() == "gloo" and part.is_cuda:  # gloo has no device gather: stage through the host
        host = part.cpu()
        hg = [torch.empty_like(host) for _ in range(world)] if rank == dst else None
        dist.gather(host, hg, dst=dst)
        if rank != dst:
            return None
        full = assemble(hg, height, world)
        return full.to(part.device) if out is None else out.copy_(full)
    if rank == dst and gathered is None:
        gathered = [torch.empty_like(part) for _ in range(world)]
    dist.gather(part, gathered if rank == dst else None, dst=dst)
    if rank != dst:
        return None
    return assemble(gathered, height, world, out)
