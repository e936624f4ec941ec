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


@pytest.mark.parametrize("world,block,expect", [(2, None, 1), (3, None, 1), (2, 8, 8), (3, 4, 4)])
def test_bench_self_launches_ranks_and_gathers(world, block, expect):
    """The selftest image has 37 rows: the auto block (balanced_block) is 1, an explicit --row-block is kept."""
    extra = [] if block is None else ["--row-block", str(block)]
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--launcher-selftest", *extra],
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res == {"launcher_selftest": True, "n_gpus": world, "parallelism": f"rows{world}", "row_block": expect,
                   "verify_gather_bitwise": True}


def test_balanced_block_deals_equal_shares():
    from hrt.parallel import balanced_block, rows_of

    assert [balanced_block(1080, n) for n in (1, 2, 3, 4, 8)] == [8, 4, 8, 2, 1]
    assert [balanced_block(2160, n) for n in (1, 2, 4, 8)] == [8, 8, 4, 2]
    for h in (225, 720, 1080, 2160, 37):
        for n in range(1, 9):
            b = balanced_block(h, n)
            assert b in (1, 2, 4, 8)
            shares = {rows_of(k, n, h, b) for k in range(n)}
            if h % n == 0:  # an even split exists, and the chosen block finds one
                assert shares == {h // n}, (h, n, b, shares)
            assert sum(rows_of(k, n, h, b) for k in range(n)) == h
