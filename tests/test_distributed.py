"""Multi-rank path on CPU (gloo, world size 2 and 3): row-tile partition + the single gather.

Each rank renders its rows with the oracle (global coordinates, as the GPU renderer does with
rt_params.row0/row_step/row_block: single interleaved rows, or the tile-aligned 8-row blocks dealt round-robin
that bench.py uses), hrt.parallel.gather_image assembles them on rank 0, and the result must equal a
single-rank render bit for bit. The GPU version of the same partition is covered by
tests/test_gpu_parity.py::test_row_partition_matches_full_image; bench.py uses the same gather over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, block, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    for p in (root, root / "hello-raytracing_amd", root / "tests"):
        sys.path.insert(0, str(p))
    import scenes
    from hrt.parallel import gather_image, max_rows, rank_params, rows_of

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sd = scenes.golden_scene("complex_scene", 40, 29)  # 29 rows: uneven split
        sd.frames = 3
        n = rows_of(rank, world, sd.height, block)
        p = rank_params(rank, world, block)
        img, _ = scenes.oracle_render(sd, rows=(p["row0"], p["row_step"], n, p["row_block"]), threads=1)
        part = torch.zeros((max_rows(world, sd.height, block), sd.width, 3), dtype=torch.float32)
        part[:n] = torch.from_numpy(img)
        full = gather_image(part, sd.height, dist, rank, world, dst=0, block=block)
        if rank == 0:
            q.put(full.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,block", [(2, 1), (3, 1), (2, 8), (3, 8)])
def test_row_tiles_gather_equals_single_rank_render(world, block):
    import scenes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, block, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd = scenes.golden_scene("complex_scene", 40, 29)
    sd.frames = 3
    ref, _ = scenes.oracle_render(sd, threads=1)
    np.testing.assert_array_equal(full.view(np.uint32), ref.view(np.uint32))


def test_rows_of_partition_covers_every_row_once():
    from hrt.parallel import rank_rows, rows_of
    for h in (1, 7, 29, 1080, 2160):
        for w in (1, 2, 3, 4, 8):
            for block in (1, 8):
                if block * (w - 1) >= h:
                    continue  # a rank would own no row (rt_set_params rejects row0 >= height)
                seen = sorted(int(r) for k in range(w) for r in rank_rows(k, w, h, block))
                assert seen == list(range(h)) and sum(rows_of(k, w, h, block) for k in range(w)) == h
    assert list(range(1, 29, 3)) == list(rank_rows(1, 3, 29, 1))


def test_blocked_rows_are_whole_tiles_dealt_round_robin():
    """8-row blocks: rank r of 8 owns tile rows r, r+8, ... of the 1080p image (17 or 16 of 135), each 8 rows
    contiguous, so the renderer's 8x8 tiles (local rows 8k..8k+7) are compact image tiles."""
    from hrt.parallel import rank_rows, rows_of
    counts = [rows_of(k, 8, 1080, 8) for k in range(8)]
    assert counts == [136] * 7 + [128]
    for k in range(8):
        rows = rank_rows(k, 8, 1080, 8).reshape(-1, 8)
        assert (rows[:, 0] % 8 == 0).all() and (rows[:, 0] // 8 % 8 == k).all()
        assert (rows - rows[:, :1] == np.arange(8)).all()


def test_oracle_blocked_rows_equal_full_render_rows():
    """The oracle's row_block mapping (the renderer's) picks exactly those rows of the full render."""
    import scenes
    from hrt.parallel import rank_params, rank_rows
    sd = scenes.golden_scene("lambertian_materials", 24, 21)
    sd.frames = 2
    full, _ = scenes.oracle_render(sd, threads=1)
    for world, rank in ((2, 1), (3, 2), (2, 0)):
        rows = rank_rows(rank, world, sd.height, 4)
        p = rank_params(rank, world, 4)
        img, _ = scenes.oracle_render(sd, rows=(p["row0"], p["row_step"], len(rows), 4), threads=1)
        np.testing.assert_array_equal(img.view(np.uint32), full[rows].view(np.uint32))
