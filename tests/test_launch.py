"""bench.py's multi-rank path without an external launcher (CPU, gloo).

`python bench.py --gpus N` with no WORLD_SIZE re-runs itself as N ranks through torch.distributed.run
(hrt.launch.spawn_ranks) before any GPU call; `--launcher-selftest` drives exactly that path — self-launch,
process group, interleaved row bands, hrt.parallel.gather_image on rank 0 — with the renderer replaced by a
row-index fill, so it runs on a CPU-only host.
"""
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_needs_self_launch():
    from hrt.launch import launch_command, needs_self_launch

    assert needs_self_launch(2, env={})
    assert not needs_self_launch(1, env={})
    assert not needs_self_launch(8, env={"WORLD_SIZE": "8"})
    cmd = launch_command(4, "bench.py", ["--gpus", "4"], port=29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-3:] == ["bench.py", "--gpus", "4"]


@pytest.mark.parametrize("world", [2, 3, 6])
def test_bench_self_launches_ranks_and_gathers(world):
    """The self-launched multi-rank path on CPU (gloo): the gather reassembles the image bit for bit, and the JSON
    line carries what the driver's one 8-GPU run needs to be diagnosed: every rank's rows,
    elapsed / trace / gather times and rays, the gather's own time, the slowest rank, and the destination rank's
    check of the gathered image's position-dependent checksum against the sum of the ranks' local ones. World 6
    leaves the last rank without rows (37 rows in 8-row blocks), which must not break the gather."""
    from hrt.parallel import rank_rows

    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--launcher-selftest"],
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert {k: res[k] for k in ("launcher_selftest", "n_gpus", "parallelism", "row_block", "verify_gather_bitwise")} == \
        {"launcher_selftest": True, "n_gpus": world, "parallelism": f"rows{world}", "row_block": 8,
         "verify_gather_bitwise": True}
    assert res["gather_checksum_ok"] is True
    ranks = res["ranks"]
    assert [d["rank"] for d in ranks] == list(range(world))
    assert [d["rows"] for d in ranks] == [len(rank_rows(k, world, 37, 8)) for k in range(world)]
    assert sum(d["rows"] for d in ranks) == 37
    for d in ranks:
        assert set(d) == {"rank", "rows", "elapsed_s", "trace_ms_per_step", "gather_ms_per_step", "rays_per_step"}
        assert d["gather_ms_per_step"] >= 0.0
    assert res["gather_ms_per_step"] == max(d["gather_ms_per_step"] for d in ranks)
    assert 0 <= res["slowest_rank"] < world


def test_image_checksum_catches_misplaced_rows():
    """hrt.parallel.image_checksum is additive over disjoint row sets and sees a row in the wrong place."""
    import numpy as np
    import torch

    from hrt.parallel import assemble, image_checksum, max_rows, rank_rows

    H, W, world = 29, 7, 3
    img = torch.from_numpy(np.random.default_rng(5).random((H, W, 3), dtype=np.float32))
    parts, total = [], 0
    for k in range(world):
        rows = rank_rows(k, world, H, 8)
        band = torch.zeros((max_rows(world, H, 8), W, 3), dtype=torch.float32)
        band[: len(rows)] = img[torch.from_numpy(rows)]
        parts.append(band)
        total += image_checksum(band, rows, W)
    full = image_checksum(img, range(H), W)
    assert (total - full) % 2**64 == 0
    assert torch.equal(assemble(parts, H, world, block=8), img)
    swapped = img.clone()
    swapped[[3, 4]] = img[[4, 3]]
    assert (total - image_checksum(swapped, range(H), W)) % 2**64 != 0
    flipped = img.clone()
    flipped.view(torch.int32)[10, 2, 1] ^= 1  # one bit of one word
    assert (total - image_checksum(flipped, range(H), W)) % 2**64 != 0
