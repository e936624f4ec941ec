"""Multi-rank path on CPU (gloo, world size 2 and 3): row-tile partition + the single gather.

Each rank renders its interleaved rows with the oracle (global coordinates, as the GPU renderer does with
rt_params.row0/row_step), hrt.parallel.gather_image assembles them on rank 0, and the result must equal a
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


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    for p in (root, root / "hello-raytracing_amd", root / "tests"):
        sys.path.insert(0, str(p))
    import scenes
    from hrt.parallel import gather_image, rows_of

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sd = scenes.golden_scene("complex_scene", 40, 29)  # 29 rows: uneven split
        sd.frames = 3
        n = rows_of(rank, world, sd.height)
        img, _ = scenes.oracle_render(sd, rows=(rank, world, n), threads=1)
        max_rows = -(-sd.height // world)
        part = torch.zeros((max_rows, sd.width, 3), dtype=torch.float32)
        part[:n] = torch.from_numpy(img)
        full = gather_image(part, sd.height, dist, rank, world, dst=0)
        if rank == 0:
            q.put(full.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_tiles_gather_equals_single_rank_render(world):
    import scenes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
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
    from hrt.parallel import rows_of
    for h in (1, 7, 1080, 2160):
        for w in (1, 2, 3, 4, 8):
            seen = sorted(r for k in range(w) for r in range(k, h, w))
            assert seen == list(range(h)) and sum(rows_of(k, w, h) for k in range(w)) == h
