"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/build/liboracle.so (rt_oracle.c).

The CPU restatement of the reference's WGSL ray loop. Imported only by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, as the checker / timed CPU baseline — never by the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "liboracle.so"

MODE_SPHERE, MODE_TRIS, MODE_MIXED = 0, 1, 2


class OParams(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("width", "height", "mode", "bounces", "ema_cap", "frame0", "time0",
                                          "dtime", "frames", "x0", "nx", "row0", "row_step", "nrows",
                                          "row_block", "step_cap")]


_libs: dict = {}


def build() -> None:
    subprocess.run(["make", "-s", "-C", os.fspath(HERE)], check=True)


def lib(contract: int = 0) -> C.CDLL:
    """The oracle library; contract 1-5 = the float-contract study variants (rt_oracle.c ORACLE_CONTRACT)."""
    if contract not in _libs:
        path = LIB if contract == 0 else HERE / "build" / f"liboracle_c{contract}.so"
        if not path.exists() or (HERE / "rt_oracle.c").exists() and path.stat().st_mtime < (HERE / "rt_oracle.c").stat().st_mtime:
            subprocess.run(["make", "-s", "-C", os.fspath(HERE), "all" if contract == 0 else "contracts"], check=True)
        L = C.CDLL(os.fspath(path))
        L.oracle_render.restype = C.c_uint64
        L.oracle_render.argtypes = [C.POINTER(OParams), C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                    C.POINTER(C.c_uint64)]
        L.oracle_sizeof.restype = C.c_uint32
        L.oracle_sizeof.argtypes = [C.c_int]
        assert [L.oracle_sizeof(i) for i in range(6)] == [80, 32, 48, 32, 64, C.sizeof(OParams)]
        _libs[contract] = L
    return _libs[contract]


def render(*, width: int, height: int, mode: int, camera: np.ndarray, frames: int, time0: int = 1000,
           dtime: int = 10, frame0: int = 0, bounces: int | None = None, ema_cap: int = 1000,
           spheres: np.ndarray | None = None, min_sphere_slots: int | None = None, bvh=None,
           rows=None, x0: int = 0, nx: int | None = None, image: np.ndarray | None = None,
           threads: int = 0, step_cap: int = 600, contract: int = 0):
    """Render `frames` frames (time0 + f*dtime, frame_count frame0 + f) of a scene.

    spheres: SPHERE_DTYPE array (zero slots appended up to min_sphere_slots, default 100 in sphere mode
    like the reference's 100-slot buffer); bvh: (sizes, nodes, triangles, materials) from Tree.view().
    rows: (row0, row_step, nrows[, row_block]) subset of rows (global coordinates), default all rows; with
    row_block b > 1 local row k is row0 + (k // b) * row_step * b + k % b (rt_params.row_block).
    step_cap: the reference walk's 600-step cap (shader_tris.wgsl:274); 0 = uncapped (only to check the
    opt-in SAH triangle walk, which has no cap).
    Returns (image[nrows, nx, 3] float32, queries).
    """
    if bounces is None:
        bounces = 10 if mode == MODE_SPHERE else 5
    if min_sphere_slots is None:
        min_sphere_slots = 100 if mode == MODE_SPHERE else 0
    row0, row_step, nrows, row_block = (tuple(rows) + (1,))[:4] if rows is not None else (0, 1, height, 1)
    nx = width - x0 if nx is None else nx
    p = OParams(width, height, mode, bounces, ema_cap, frame0, time0, dtime, frames, x0, nx, row0, row_step, nrows,
                row_block, step_cap)
    sph_ptr, nslots, keep = None, 0, []
    if mode != MODE_TRIS:
        sp = spheres if spheres is not None else np.zeros(0, dtype=np.uint8)
        n = len(sp)
        nslots = max(n, min_sphere_slots)
        buf = np.zeros(nslots * 48, dtype=np.uint8)
        if n:
            buf[: n * 48] = np.frombuffer(np.ascontiguousarray(sp).tobytes(), dtype=np.uint8)
        keep.append(buf)
        sph_ptr = buf.ctypes.data
    sizes_p = nodes_p = tris_p = mats_p = None
    if mode != MODE_SPHERE and bvh is not None:
        sizes, nodes, tris, mats = bvh
        sz = np.array(sizes, dtype=np.uint32)
        nodes, tris, mats = (np.ascontiguousarray(a) for a in (nodes, tris, mats))
        keep += [sz, nodes, tris, mats]
        sizes_p, nodes_p, tris_p, mats_p = sz.ctypes.data, nodes.ctypes.data, tris.ctypes.data, mats.ctypes.data
    elif mode != MODE_SPHERE:
        sz = np.zeros(2, dtype=np.uint32)
        keep.append(sz)
        sizes_p = sz.ctypes.data
    if image is None:
        image = np.zeros((nrows, nx, 3), dtype=np.float32)
    else:
        image = np.ascontiguousarray(image, dtype=np.float32).copy()
        assert image.shape == (nrows, nx, 3)
    cam = np.ascontiguousarray(camera).tobytes()
    if threads <= 0:  # explicit: importing torch can leave the OpenMP default at one thread
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    counts = (C.c_uint64 * 4)()
    q = lib(contract).oracle_render(C.byref(p), cam, sph_ptr, nslots, sizes_p, nodes_p, tris_p, mats_p,
                            image.ctypes.data, threads, counts)
    last_counts.update(rays=counts[0], node_tests=counts[1], tri_tests=counts[2], capped_walks=counts[3])
    return image, int(q)


# {rays, node_tests, tri_tests} of the last render() call (triangle-program work counters)
last_counts: dict = {}
