"""The multi-GPU gather over RCCL, as far as one GPU can take it (bench.py's nccl branch).

The driver's 8-GPU run is the only place where ranks > 1 meet over xGMI; the gloo tests (tests/test_distributed.py)
cover the partition and the gather's logic on CPU. Here one child process opens a one-rank `nccl` (RCCL) process group
bound to cuda:0 exactly as bench.py does, renders its row band with the HIP renderer, and runs the path's collectives
on the device tensors: the `dist.gather` of hrt.parallel.gather_image's nccl branch (called with the band twice, as
if from two ranks, is not possible with one GPU: RCCL refuses two ranks on one device) and the all-reduce that
bench.py's rank reports use. The gathered band must equal the rendered one bit for bit.
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

import hrt

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import sys
sys.path[:0] = [{root!r}, {pkg!r}, {tests!r}]
import torch, torch.distributed as dist
import hrt, scenes
from hrt.parallel import assemble, max_rows, rank_params, rows_of
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
sd = scenes.config_c3(96, 64, 4)
r = scenes.make_renderer(sd)
r.set_params(**rank_params(0, 1, 8))
r.draw_frames(sd.frames, 1000, 10)
part = torch.zeros((max_rows(1, sd.height, 8), sd.width, 3), dtype=torch.float32, device="cuda")
r.copy_image_to_device(part.data_ptr(), rows_of(0, 1, sd.height, 8) * sd.width * 3)
torch.cuda.synchronize()
out = [torch.empty_like(part)]
dist.gather(part, out, dst=0)
full = assemble(out, sd.height, 1, block=8)
assert torch.equal(full.view(torch.int32), part.view(torch.int32)), "gathered band differs"
import numpy as np
assert np.array_equal(full.cpu().numpy().view(np.uint32), r.read_image().view(np.uint32)), "band differs from the image"
s = torch.tensor([float(part.double().sum().item())], dtype=torch.float64, device="cuda")
dist.all_reduce(s)
torch.cuda.synchronize()
dist.destroy_process_group()
print("rccl ok", torch.cuda.get_device_name(0), float(s.item()))
"""


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_one_rank_rccl_gather_of_a_rendered_band():
    if hrt.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on an MI355X box (there is no CPU fallback)")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    code = CHILD.format(root=str(ROOT), pkg=str(ROOT / "hello-raytracing_amd"), tests=str(ROOT / "tests"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert "rccl ok" in p.stdout, p.stdout[-2000:]
