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
    fields = {"rank", "rows", "elapsed_s", "trace_ms_per_step", "gather_ms_per_step", "rays_per_step", "device", "pci",
              "torch_device", "torch_pci"}
    # the headline leg (37 rows) and the C5 leg of a multi-rank run (53 rows here)
    for blk, H in ((res, 37), (res["c5"], 53)):
        assert blk["gather_checksum_ok"] is True
        ranks = blk["ranks"]
        assert [d["rank"] for d in ranks] == list(range(world))
        assert [d["rows"] for d in ranks] == [len(rank_rows(k, world, H, 8)) for k in range(world)]
        assert sum(d["rows"] for d in ranks) == H
        for d in ranks:
            assert set(d) == fields
            assert d["gather_ms_per_step"] >= 0.0
            # no GPU in the self-test: the renderer / torch device fields are present and empty
            assert (d["device"], d["pci"], d["torch_device"], d["torch_pci"]) == (-1, None, -1, None)
        assert blk["gather_ms_per_step"] == max(d["gather_ms_per_step"] for d in ranks)
        assert 0 <= blk["slowest_rank"] < world
        assert blk["device_check_ok"] is None and blk["device_error"] is None
    assert res["c5"]["config"]["id"] == "c5" and res["c5"]["verify_gather_bitwise"] is True


def _report(world, devices, pcis, tdevices=None, tpcis=None):
    return [{"rank": k, "rows": 1, "elapsed_s": 0.0, "trace_ms": 0.0, "gather_ms": 0.0, "queries": 0, "checksum": 0,
             "device": devices[k], "pci": pcis[k], "torch_device": (tdevices or devices)[k],
             "torch_pci": (tpcis or pcis)[k]} for k in range(world)]


def test_device_check_fails_the_line_on_a_wrong_or_shared_gpu():
    """bench.device_check: each rank's renderer must draw on torch's current device, and under RCCL
    no two ranks may share a GPU. The cases a one-GPU box cannot produce, on synthetic reports."""
    import bench

    pci = [bench.pci_code((0, 0x05 + 0x10 * k, 0)) for k in range(4)]
    assert bench.device_check(_report(4, [0, 1, 2, 3], pci), True) == (True, None)
    # every renderer on GPU 0 while torch moved each rank to its own GPU (two HIP runtimes)
    ok, msg = bench.device_check(_report(4, [0, 0, 0, 0], [pci[0]] * 4, [0, 1, 2, 3], pci), True)
    assert ok is False and "ranks [1, 2, 3]" in msg
    # two ranks on one GPU (both consistent with torch): fails under RCCL, allowed in a gloo rehearsal
    shared = [pci[0], pci[1], pci[1], pci[3]]
    ok, msg = bench.device_check(_report(4, [0, 1, 1, 3], shared), True)
    assert ok is False and "0000:15:00" in msg and "[1, 2]" in msg
    assert bench.device_check(_report(4, [0, 1, 1, 3], shared), False) == (True, None)
    assert bench.pci_str(bench.pci_code((1, 0xC3, 2))) == "0001:c3:02"


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
