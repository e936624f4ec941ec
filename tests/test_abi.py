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


TESTING_HEADER = (ROOT / "include" / "hrt_testing.h").read_text()


def declared_functions(text=HEADER):
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(rt_\w+)\s*\(", text, re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("rt_create", "rt_set_camera", "rt_set_spheres", "rt_set_bvh", "rt_draw", "rt_draw_frames",
                 "rt_read_image", "rt_host_camera_new", "rt_host_tree_build", "rt_host_render_ppm"):
        assert must in names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (rt_\w+)", out))
    missing = [n for n in declared_functions() + declared_functions(TESTING_HEADER) if n not in exported]
    assert not missing, missing
    assert set(_lib.SIGNATURES) == set(declared_functions())
    assert set(_lib.TESTING_SIGNATURES) == set(declared_functions(TESTING_HEADER))
    # the public header declares no test-only entry point, and rt_params carries no fault-injection field
    assert not set(declared_functions(TESTING_HEADER)) & set(declared_functions())
    assert "fail_alloc" not in HEADER and "ring_slots_max" not in HEADER
    L = hrt.lib()
    for n in declared_functions():
        assert getattr(L, n) is not None


def test_bvh_size_rules_without_a_device():
    """rt_set_bvh's size rules (the walks' buffer descriptors take 32-bit byte sizes and offsets, so
    n x 32 B and m x 64 B must stay below 4 GiB; n a power of two as Tree::build makes it), checked on the host."""
    L = hrt.lib()

    def check(n, m, n_nodes=None, n_tris=None, n_mats=1):
        sizes = (C.c_uint32 * 2)(n, m)
        return L.rt_host_check_bvh_sizes(sizes, n if n_nodes is None else n_nodes, m if n_tris is None else n_tris,
                                         n_mats)

    assert check(1024, 979) == _lib.RT_OK                              # Suzanne (tree.rs:121-124)
    assert check(16, 12) == _lib.RT_OK                                 # cube (tree.rs:107-110)
    assert check(1 << 26, (1 << 26) - 1) == _lib.RT_OK                 # the largest tree: 2 GiB of nodes, 4 GiB of tris
    assert check(1 << 27, (1 << 26) + 1) == _lib.RT_ERR_ARG            # n x 32 B would wrap a 32-bit size
    assert b"RT_MAX_TREE_NODES" in L.rt_last_error()
    assert check(1 << 26, 1 << 26) == _lib.RT_ERR_ARG                  # m x 64 B would wrap
    assert check(1000, 979) == _lib.RT_ERR_ARG                         # not a power of two
    assert check(0, 0) == _lib.RT_ERR_ARG
    assert check(1024, 979, n_nodes=1023) == _lib.RT_ERR_ARG           # sizes exceed the buffers given
    assert check(1024, 979, n_tris=978) == _lib.RT_ERR_ARG
    assert check(1024, 979, n_mats=1 << 28) == _lib.RT_ERR_ARG
    assert L.rt_host_check_bvh_sizes(None, 1, 1, 1) == _lib.RT_ERR_ARG


def test_library_reads_no_environment_knobs():
    """the product library takes every setting through rt_params / arguments, none from the environment
    (the diagnostic build, lib/libhrt_diag.so, may read HRT_RING_DUMP). libhrt.so imports no environment accessor
    (getenv, secure_getenv, environ), so no code in it can read a variable (the HIP runtime it loads reads its own
    HIP_* / HSA_* settings), and no HRT_-prefixed name is left in its strings."""
    out = subprocess.run(["nm", "-D", "--undefined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    imported = set(re.findall(r"\bU (\w+)", out))
    assert imported, out  # (the scan saw the import table: HIP runtime and libc symbols)
    assert not imported & {"getenv", "secure_getenv", "__secure_getenv", "environ", "__environ", "getenv_s"}, imported
    data = _lib.LIB_PATH.read_bytes()
    names = sorted(set(re.findall(rb"HRT_[A-Z0-9_]{2,}", data)))
    assert not names, names


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
    assert C.sizeof(hrt.RtParams) == 20 * 4
    assert C.sizeof(hrt.RtStats) == 8 + 8 + 8 + 4 + 4 + 8 + 8 + 4 + 4 + 8 + 8 + 8 + 4 + 4 + 64 + 8 + 4 + 4 + 8 + 4 + 4
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


def test_device_code_object_is_gfx950(tmp_path):
    # (objdump --offloading writes the extracted bundles next to its input: run it on a copy)
    lib = tmp_path / _lib.LIB_PATH.name
    lib.write_bytes(_lib.LIB_PATH.read_bytes())
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    text = out.stdout + out.stderr
    if "gfx950" not in text:  # older objdump: look for the bundle id string directly
        assert b"gfx950" in _lib.LIB_PATH.read_bytes()


def test_abi_version_guard():
    """rt_abi_version reports the header's version and the sizes rt_set_params / rt_get_stats copy."""
    text = (Path(__file__).resolve().parents[1] / "include" / "hrt.h").read_text()
    want = int(re.search(r"#define RT_ABI_VERSION (\d+)u", text).group(1))
    v, pb, sb = C.c_uint32(), C.c_uint32(), C.c_uint32()
    assert hrt.lib().rt_abi_version(C.byref(v), C.byref(pb), C.byref(sb)) == 0
    assert (v.value, pb.value, sb.value) == (want, C.sizeof(hrt.RtParams), C.sizeof(hrt.RtStats))
    assert hrt.lib().rt_abi_version(None, None, None) == 0


def test_hip_runtime_choice_follows_the_soname():
    """lib() preloads torch's HIP runtime only when its SONAME is the one libhrt.so needs, and says which
    runtime it chose; the ELF reader it uses sees libhrt.so's DT_NEEDED."""
    needed = _lib.elf_dynamic_names(_lib.LIB_PATH, 1)
    assert any(n.startswith("libamdhip64.so") for n in needed), needed
    hrt.lib()
    choice = _lib.HIP_RUNTIME_CHOICE
    trt = _lib._torch_hip_runtime()
    if trt is None:
        assert choice["path"] is None and "torch not installed" in choice["reason"]
    elif _lib.elf_dynamic_names(trt, 14) == [n for n in needed if n.startswith("libamdhip64")]:
        assert choice["path"] == str(trt) and "preloaded" in choice["reason"]
    else:
        assert choice["path"] is None and "does not match" in choice["reason"]
    assert len(_lib.hip_runtimes()) <= 1
