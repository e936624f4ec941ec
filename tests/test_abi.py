"""The C-ABI boundary: libhrt.so loads, exports exactly what include/hrt.h declares, and fails loudly
(no CPU fallback) when no GPU is present. CPU only; never calls compute on a GPU."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

import hrt
from hrt import _lib

ROOT = Path(__file__).resolve().parents[1]
HEADER = (ROOT / "include" / "hrt.h").read_text()


def declared_functions():
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(rt_\w+)\s*\(", HEADER, re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("rt_create", "rt_set_camera", "rt_set_spheres", "rt_set_bvh", "rt_draw", "rt_draw_frames",
                 "rt_read_image", "rt_host_camera_new", "rt_host_tree_build", "rt_host_render_ppm"):
        assert must in names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (rt_\w+)", out))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    assert set(_lib.SIGNATURES) == set(declared_functions())
    L = hrt.lib()
    for n in declared_functions():
        assert getattr(L, n) is not None


def _header_struct(name):
    """(type, field) pairs of `typedef struct name {...} name;` in include/hrt.h (comments stripped)."""
    text = (ROOT / "include" / "hrt.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), text, flags=re.S).group(1)
    return [(t, n.strip()) for t, names in re.findall(r"(uint32_t|uint64_t|double|char)\s+([\w\s,\[\]]+);", body)
            for n in names.split(",")]


def test_struct_layouts_match_header():
    ctypes_of = {"uint32_t": C.c_uint32, "uint64_t": C.c_uint64, "double": C.c_double}

    def ctype(t, f):
        m = re.fullmatch(r"(\w+)\[(\d+)\]", f)
        return (m.group(1), {"char": C.c_char}[t] * int(m.group(2))) if m else (f, ctypes_of[t])

    for py, name in ((hrt.RtParams, "rt_params"), (hrt.RtStats, "rt_stats")):
        fields = [ctype(t, f) for t, f in _header_struct(name)]
        got = [(f, t) for f, t in py._fields_]
        assert [f for f, _ in fields] == [f for f, _ in got], name
        assert [C.sizeof(t) for _, t in fields] == [C.sizeof(t) for _, t in got], name
    assert C.sizeof(hrt.RtParams) == 19 * 4
    assert C.sizeof(hrt.RtStats) == 8 + 8 + 8 + 4 + 4 + 8 + 8 + 4 + 4 + 8 + 8 + 8 + 4 + 4 + 64 + 8 + 4 + 4 + 8
    from oracle import oracle as O
    assert [O.lib().oracle_sizeof(i) for i in range(6)] == [80, 32, 48, 32, 64, C.sizeof(O.OParams)]


def test_renderer_fails_loudly_without_gpu():
    if hrt.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(hrt.RtError) as e:
        hrt.Renderer(16, 16, hrt.RT_MODE_SPHERE)
    assert e.value.code == _lib.RT_ERR_DEVICE
    assert "no CPU fallback" in str(e.value)


def test_bad_arguments_are_rejected_before_the_device():
    h = C.c_void_p()
    assert hrt.lib().rt_create(0, 16, 0, C.byref(h)) == _lib.RT_ERR_ARG
    assert hrt.lib().rt_create(16, 16, 7, C.byref(h)) == _lib.RT_ERR_ARG
    assert hrt.lib().rt_draw(None) == _lib.RT_ERR_ARG
    assert hrt.lib().rt_host_camera_new(None, None, 1.0, 0.0, 1.0, None) == _lib.RT_ERR_ARG


def test_device_code_object_is_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(_lib.LIB_PATH)],
                         capture_output=True, text=True)
    text = out.stdout + out.stderr
    if "gfx950" not in text:  # older objdump: look for the bundle id string directly
        assert b"gfx950" in _lib.LIB_PATH.read_bytes()
