"""Row-tile partition of the image across ranks and the one gather that assembles it.

SURVEY §8(e): every pixel is independent (seed = f(global x, global y, H, time)), so each rank renders a
subset of the image rows with global coordinates and one collective gather over RCCL (xGMI on one node)
brings the row bands to the destination rank, which puts the rows back in place. There is no other
data-path communication. Works with any torch.distributed backend (nccl = RCCL on GPUs, gloo on CPU for
the tests).

The partition deals BLOCKS of `block` rows round-robin: rank r of N owns rows
    8r .. 8r+7, 8(r+N) .. 8(r+N)+7, ...            (block = 8, the default of bench.py)
i.e. rt_params.row0 = block * r, row_step = N, row_block = block. With block = 8 every 8x8 tile of the
sample queue (rt_kernels.hip) is a compact tile of the image, as it is on one GPU; single interleaved
rows (block = 1) would stretch a tile over 8N image rows and cost ray coherence.
Dealing blocks round-robin keeps the cheap sky rows spread over the ranks.
"""
from __future__ import annotations

import numpy as np


def rank_params(rank: int, world: int, block: int = 1) -> dict:
    """rt_params fields of rank `rank` of `world` (Renderer.set_params(**rank_params(...)))."""
    return {"row0": block * rank, "row_step": world, "row_block": block}


def owned_rows(row0: int, row_step: int, height: int, block: int = 1) -> np.ndarray:
    """Global rows a renderer with (row0, row_step, row_block) owns, in its local row order
    (renderer.cpp local_rows_of, rt_device.hpp global_row)."""
    block = max(int(block), 1)
    if row0 >= height or row_step <= 0:
        return np.zeros(0, dtype=np.int64)
    starts = np.arange(row0, height, row_step * block, dtype=np.int64)
    rows = (starts[:, None] + np.arange(block, dtype=np.int64)[None, :]).ravel()
    return rows[rows < height]


def local_rows(row0: int, row_step: int, height: int, block: int = 1) -> int:
    return int(len(owned_rows(row0, row_step, height, block)))


def rank_rows(rank: int, world: int, height: int, block: int = 1) -> np.ndarray:
    """Global rows of rank `rank` of `world`, in its local order."""
    p = rank_params(rank, world, block)
    return owned_rows(p["row0"], p["row_step"], height, block)


def rows_of(rank: int, world: int, height: int, block: int = 1) -> int:
    """Number of rows owned by `rank`."""
    return int(len(rank_rows(rank, world, height, block)))


def max_rows(world: int, height: int, block: int = 1) -> int:
    """Rows of the largest band (the padded gather size)."""
    return max(rows_of(k, world, height, block) for k in range(world))


def assemble(parts, height: int, world: int, out=None, block: int = 1):
    """Put the rows back in place: parts[k] holds rank k's rows in its local order (padded to max_rows)."""
    import torch

    if out is None:
        out = torch.empty((height,) + tuple(parts[0].shape[1:]), dtype=parts[0].dtype, device=parts[0].device)
    for k in range(world):
        idx = rank_rows(k, world, height, block)
        if len(idx) == 0:
            continue
        if block == 1:
            out[int(idx[0])::world] = parts[k][: len(idx)]
        else:
            out[torch.from_numpy(idx).to(out.device)] = parts[k][: len(idx)]
    return out


def gather_image(part, height: int, dist, rank: int, world: int, dst: int = 0, gathered=None, out=None,
                 block: int = 1):
    """Collective: every rank passes its padded (max_rows, W, 3) band; returns the full image on `dst` (None
    elsewhere). One dist.gather — the only collective of the path."""
    import torch

    if world == 1:
        return part[:height] if out is None else out.copy_(part[:height])
    if dist.get_backend() == "gloo" and part.is_cuda:  # gloo has no device gather: stage through the host
        host = part.cpu()
        hg = [torch.empty_like(host) for _ in range(world)] if rank == dst else None
        dist.gather(host, hg, dst=dst)
        if rank != dst:
            return None
        full = assemble(hg, height, world, block=block)
        return full.to(part.device) if out is None else out.copy_(full)
    if rank == dst and gathered is None:
        gathered = [torch.empty_like(part) for _ in range(world)]
    dist.gather(part, gathered if rank == dst else None, dst=dst)
    if rank != dst:
        return None
    return assemble(gathered, height, world, out, block=block)


def image_checksum(img, rows, width: int) -> int:
    """Position-dependent checksum of image rows: sum over the f32 words w at global flat index g of
    w * (2g + 1) (mod 2^64, as a signed int64). `img` holds the rows `rows` (global indices, local order) of an
    image `width` pixels wide, 3 words per pixel (extra padding rows beyond len(rows) are ignored). Additive over
    disjoint row sets, so the gathered image's checksum on the destination rank equals the sum of the ranks' local
    checksums exactly when every rank's words arrived at the right place (bench.py, multi-rank runs)."""
    import torch

    n = len(rows)
    if n == 0:
        return 0
    words = img[:n].reshape(n, width * 3).contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    r = torch.as_tensor(np.asarray(rows, dtype=np.int64), device=words.device)[:, None]
    g = r * (width * 3) + torch.arange(width * 3, dtype=torch.int64, device=words.device)[None, :]
    return int((words * (2 * g + 1)).sum().item())

