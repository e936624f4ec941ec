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


@pytest.mark.parametrize("world", [2, 3])
def test_bench_self_launches_ranks_and_gathers(world):
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--launcher-selftest"],
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res == {"launcher_selftest": True, "n_gpus": world, "parallelism": f"rows{world}", "row_block": 8,
                   "verify_gather_bitwise": True}
