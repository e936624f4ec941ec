"""One process per GPU without an external launcher.

`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) re-runs the same script as N ranks of
one node through `torch.distributed.run` in a child process — started before the parent makes any HIP
call, so the parent never holds a GPU context — and exits with the child's status. Each rank then reads
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* like a driver-launched rank (row tiles, one
RCCL gather). The rendezvous is on 127.0.0.1 (the container hostname may not resolve).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def needs_self_launch(nprocs: int, env=None) -> bool:
    """True when N > 1 ranks are wanted and this process is not already one of them."""
    env = os.environ if env is None else env
    return nprocs > 1 and "WORLD_SIZE" not in env


def launch_command(nprocs: int, script: str, argv: list[str], port: int | None = None) -> list[str]:
    """The torch.distributed.run command line the driver itself would use for N ranks of one node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nprocs}",
            "--master-addr", "127.0.0.1", "--master-port", str(port or free_port()), script, *argv]


def spawn_ranks(nprocs: int, script: str, argv: list[str], timeout: float | None = None) -> int:
    """Run `script argv` as `nprocs` ranks (child process); returns its exit code. The parent must not
    have touched the GPU (exec-ing or forking a GPU-initialised process is unsafe on this pool)."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC: RCCL / tensor sharing across ranks
    env.setdefault("OMP_NUM_THREADS", "1")
    proc = subprocess.run(launch_command(nprocs, script, argv), env=env, timeout=timeout)
    return proc.returncode
