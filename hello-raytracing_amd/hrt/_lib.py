"""ctypes binding of lib/libhrt.so (declared in include/hrt.h).

The library is built in-tree by `make -C hello-raytracing_amd` (or __graft_entry__.build()). Loading it
never touches the GPU; renderer calls fail with RT_ERR_DEVICE on a host without a gfx950 device —
there is no CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent  # hello-raytracing_amd/
# HRT_LIB may name the diagnostic build (lib/libhrt_diag.so, relative to the package) for timing studies.
LIB_PATH = PKG_ROOT / os.environ.get("HRT_LIB", "lib/libhrt.so")

RT_OK = 0
RT_ERR_ARG = -1
RT_ERR_DEVICE = -2
RT_ERR_ALLOC = -3
RT_ERR_STATE = -4
RT_ERR_PARSE = -5
RT_ERR_COMPARE = -6

RT_MODE_SPHERE = 0
RT_MODE_TRIS = 1
RT_MODE_MIXED = 2
RT_SCHEDULE_AUTO, RT_SCHEDULE_TILES, RT_SCHEDULE_QUEUE = 0, 1, 2
RT_FOLD_AUTO, RT_FOLD_BUFFER, RT_FOLD_RING = 0, 1, 2


class RtParams(C.Structure):
    _fields_ = [
        ("bounces", C.c_uint32),
        ("ema_cap", C.c_uint32),
        ("min_sphere_slots", C.c_uint32),
        ("row0", C.c_uint32),
        ("row_step", C.c_uint32),
        ("frames_per_launch", C.c_uint32),
        ("variant", C.c_uint32),
        ("schedule", C.c_uint32),
        ("queue_budget_mb", C.c_uint32),
        ("job_frames", C.c_uint32),
        ("tri_bvh", C.c_uint32),
        ("suspend_below", C.c_uint32),
        ("row_block", C.c_uint32),
        ("fold", C.c_uint32),
        ("heap_lds", C.c_uint32),
        ("steal", C.c_uint32),
        ("tail_split", C.c_uint32),
        ("count_tests", C.c_uint32),
    ]


class RtStats(C.Structure):
    _fields_ = [
        ("queries", C.c_uint64),
        ("samples", C.c_uint64),
        ("kernel_ms", C.c_double),
        ("launches", C.c_uint32),
        ("local_rows", C.c_uint32),
        ("box_tests", C.c_uint64),
        ("sphere_tests", C.c_uint64),
        ("variant", C.c_uint32),
        ("schedule", C.c_uint32),
        ("node_tests", C.c_uint64),
        ("tri_tests", C.c_uint64),
        ("trace_ms", C.c_double),
        ("trace_launches", C.c_uint32),
        ("suspend_below", C.c_uint32),
        ("kernel", C.c_char * 64),
        ("fold_bytes", C.c_uint64),
        ("fold_ring", C.c_uint32),
        ("launch_frames", C.c_uint32),
        ("device_bytes", C.c_uint64),
    ]


# Every exported symbol of include/hrt.h with its ctypes signature.
_P = C.c_void_p
_U32 = C.c_uint32
_PU32 = C.POINTER(C.c_uint32)
_PF = C.POINTER(C.c_float)
SIGNATURES = {
    "rt_create": (C.c_int, [_U32, _U32, C.c_int, C.POINTER(_P)]),
    "rt_destroy": (C.c_int, [_P]),
    "rt_get_params": (C.c_int, [_P, C.POINTER(RtParams)]),
    "rt_set_params": (C.c_int, [_P, C.POINTER(RtParams)]),
    "rt_set_camera": (C.c_int, [_P, C.c_char_p]),
    "rt_set_spheres": (C.c_int, [_P, C.c_char_p, _U32]),
    "rt_set_bvh": (C.c_int, [_P, _PU32, _P, _U32, _P, _U32, _P, _U32]),
    "rt_set_time": (C.c_int, [_P, _U32]),
    "rt_set_frame_count": (C.c_int, [_P, _U32]),
    "rt_get_frame_count": (C.c_int, [_P, _PU32]),
    "rt_draw": (C.c_int, [_P]),
    "rt_draw_frames": (C.c_int, [_P, _U32, _U32, _U32]),
    "rt_read_image": (C.c_int, [_P, _PF, C.c_size_t]),
    "rt_write_image": (C.c_int, [_P, _PF, C.c_size_t]),
    "rt_copy_image_to_device": (C.c_int, [_P, _P, C.c_size_t]),
    "rt_reset_frame_count": (C.c_int, [_P]),
    "rt_resize": (C.c_int, [_P, _U32, _U32]),
    "rt_synchronize": (C.c_int, [_P]),
    "rt_release_scratch": (C.c_int, [_P]),
    "rt_get_stats": (C.c_int, [_P, C.POINTER(RtStats)]),
    "rt_get_raw_counters": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_int]),
    "rt_diagnostic_build": (C.c_int, []),
    "rt_check_exact_math": (C.c_int, [C.c_uint64, C.c_uint32, C.POINTER(C.c_uint64)]),
    "rt_get_wave_trace": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_size_t]),
    "rt_last_error": (C.c_char_p, []),
    "rt_device_count": (C.c_int, []),
    "rt_build_info": (C.c_char_p, []),
    "rt_host_check_bvh_sizes": (C.c_int, [_PU32, _U32, _U32, _U32]),
    "rt_host_camera_new": (C.c_int, [_PF, _PF, C.c_float, C.c_float, C.c_float, C.c_char_p]),
    "rt_host_mesh_load_obj": (C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.POINTER(_P)]),
    "rt_host_mesh_counts": (C.c_int, [_P, _PU32, _PU32]),
    "rt_host_mesh_destroy": (C.c_int, [_P]),
    "rt_host_tree_new": (C.c_int, [C.POINTER(_P)]),
    "rt_host_tree_add_mesh": (C.c_int, [_P, _P]),
    "rt_host_tree_build": (C.c_int, [_P]),
    "rt_host_tree_build_threads": (C.c_int, [_P, C.c_int]),
    "rt_host_tree_view": (
        C.c_int,
        [_P, _PU32, C.POINTER(_P), _PU32, C.POINTER(_P), _PU32, C.POINTER(_P), _PU32],
    ),
    "rt_host_tree_destroy": (C.c_int, [_P]),
    "rt_host_render_ppm": (C.c_int, [_PF, _U32, _U32, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "rt_host_compare_ppm": (
        C.c_int,
        [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_float, C.POINTER(C.c_int), _PF],
    ),
}

# include/hrt_testing.h: test-only entry points (fault injection), not part of the drop-in surface.
TESTING_SIGNATURES = {
    "rt_testing_set_faults": (C.c_int, [_P, _U32, _U32]),
}

_lib = None


class RtError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str = ""):
        super().__init__(f"{where} failed with status {code}: {msg}")
        self.code = code


def lib() -> C.CDLL:
    """Load libhrt.so once. Raises if it was not built (no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make -C {PKG_ROOT}` "
                "(or __graft_entry__.build()); the renderer has no Python/CPU fallback"
            )
        L = C.CDLL(os.fspath(LIB_PATH))
        for name, (res, args) in {**SIGNATURES, **TESTING_SIGNATURES}.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, where: str) -> None:
    if rc != RT_OK:
        msg = lib().rt_last_error()
        raise RtError(rc, where, msg.decode() if msg else "")
