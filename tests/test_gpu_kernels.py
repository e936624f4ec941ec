"""Every kernel instantiation in lib/libhrt.so is reached through rt_params and renders the oracle's bits; and the
triangle / mixed programs' primary rays with d = 0.

test_every_instantiation_is_reached: the product library holds one instantiation per (program, sphere scan, heap-top
configuration, stealing, counting, SAH walk) combination the launcher can pick (rt_kernels.hip hrt_launch_trace /
hrt_launch_render). Each case below selects one through the public rt_params and draws a small scene; the set of
kernels the draws report (rt_stats.kernel) must equal the set in the code object (no instantiation that
no default or test path reaches), and each draw must match the oracle bit for bit with its ray count (the opt-in SAH
walk, non-parity by contract, against the uncapped oracle).
"""
import re
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import hrt
import scenes
from hrt import PI, Camera, Vec3, f32

pytestmark = pytest.mark.gpu

LIB = Path(__file__).resolve().parents[1] / "hello-raytracing_amd" / "lib" / "libhrt.so"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if hrt.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on an MI355X box (there is no CPU fallback)")


def library_kernels() -> set:
    """Demangled names of the ray-tracing kernels in the code object (their kernel-descriptor symbols)."""
    data = LIB.read_bytes()
    syms = sorted({m.decode() for m in re.findall(rb"_Z[0-9A-Za-z_]*k_(?:trace|render)[0-9A-Za-z_]*\.kd", data)})
    out = subprocess.run(["c++filt"], input="\n".join(s[:-3] for s in syms), capture_output=True, text=True,
                         check=True).stdout.split("\n")
    return {re.sub(r"^void ", "", s.split("(")[0]) for s in out if s.strip()}


def _deep_spheres():
    """Two seeded cover scenes: a culling BVH of > 192 nodes (k_trace_split without LDS nodes)."""
    return np.concatenate([scenes.rtiow_spheres(42), scenes.rtiow_spheres(7)])


def _cases():
    c3 = scenes.config_c3(40, 24, 3)
    deep = scenes.config_c3(40, 24, 3)
    deep.spheres = _deep_spheres()
    c4 = scenes.config_c4(40, 24, 3)  # 1 sphere: the simple scan
    defer = scenes.config_c4(40, 24, 3)
    defer.spheres = np.concatenate([defer.spheres, scenes.rtiow_spheres()[1:12]])  # 12 slots: the deferred scan
    bvh = scenes.config_c4(40, 24, 3)
    bvh.spheres = np.concatenate([bvh.spheres, scenes.rtiow_spheres()[1:60]])  # 60 slots: the culling BVH
    suz = hrt.SceneTris.new_suzane(40, 24)
    tris = scenes.SceneDef("suzane", hrt.RT_MODE_TRIS, 40, 24, suz.camera, bvh=suz.tris_bvh.view(), frames=3)
    Q, T = hrt.RT_SCHEDULE_QUEUE, hrt.RT_SCHEDULE_TILES
    cases = []
    for sd in (c3, deep):
        for steal in (1, 2):
            for count in (0, 1):
                for packet in ((1, 2) if sd is c3 else (0,)):  # (the packet walk needs the LDS nodes: not the deep tree)
                    cases.append((sd, dict(schedule=Q, steal=steal, count_tests=count, packet=packet)))
    for v in (1, 3):
        cases.append((c3, dict(schedule=Q, variant=v, steal=1)))
    for v in (1, 3, 4):
        cases.append((c3, dict(schedule=T, variant=v)))
    for sd in (tris, c4, defer, bvh):
        for heap_lds in (1, 2):
            for steal in (1, 2):
                cases.append((sd, dict(schedule=Q, heap_lds=heap_lds, steal=steal)))
        for tri_bvh in (0, 1):
            cases.append((sd, dict(schedule=T, tri_bvh=tri_bvh)))
        cases.append((sd, dict(schedule=Q, tri_bvh=1)))
    return cases


def test_every_instantiation_is_reached():
    if shutil.which("c++filt") is None:
        pytest.skip("needs c++filt")
    want = library_kernels()
    assert len(want) >= 30, want
    seen = {}
    for sd, params in _cases():
        r = scenes.make_renderer(sd)
        r.set_params(**params)
        r.draw_frames(sd.frames, 1000, 10)
        img, st = r.read_image(), r.stats()
        k = st.kernel.decode()
        seen.setdefault(k, (sd.name, params))
        ref, q = scenes.oracle_render(sd, step_cap=0 if params.get("tri_bvh") else 600)
        what = f"{sd.name} {params} -> {k}"
        np.testing.assert_array_equal(img.view(np.uint32), ref.view(np.uint32), err_msg=what)
        assert st.queries == q, what
    missing = want - set(seen)
    extra = set(seen) - want
    assert not missing, f"instantiations no case reaches: {sorted(missing)}"
    assert not extra, f"kernels reported but not in the library: {sorted(extra)}"


@pytest.mark.parametrize("blur", [0.0, 0.3])
@pytest.mark.parametrize("mode", ["tris", "mixed"])
def test_focal_length_zero_primary_rays(mode, blur):
    """Camera focal_length 0 (and blur 0): every primary ray of the triangle / mixed programs has d = 0
    (make_ray, shader_tris.wgsl:136-148: f = eye, g = f - o = (0, 0, 0, -1), d = (g / |g|).xyz = 0); the reference
    traces it (1 / d = inf in the node tests). The frame-block refill once used d = 0 as its 'pixel outside the
    image' marker and skipped these samples; now an in-image mask decides. Queue (both heap-top
    configurations) and tiles against the oracle, with a ragged edge tile."""
    suz = hrt.SceneTris.new_suzane(44, 27)
    cam = Camera.new(Vec3(0.0, 0.5, 3.0), Vec3(0.0, 0.0, -1.0), 0.0, blur, PI * f32(0.3))
    if mode == "tris":
        sd = scenes.SceneDef("suzane-focal0", hrt.RT_MODE_TRIS, 44, 27, cam, bvh=suz.tris_bvh.view(), frames=3)
    else:
        sd = scenes.config_c4(44, 27, 3)
        sd.camera = cam
    ref, q = scenes.oracle_render(sd)
    for params in (dict(schedule=hrt.RT_SCHEDULE_QUEUE), dict(schedule=hrt.RT_SCHEDULE_QUEUE, heap_lds=1),
                   dict(schedule=hrt.RT_SCHEDULE_QUEUE, steal=2), dict(schedule=hrt.RT_SCHEDULE_TILES)):
        r = scenes.make_renderer(sd)
        r.set_params(**params)
        r.draw_frames(sd.frames, 1000, 10)
        img, st = r.read_image(), r.stats()
        np.testing.assert_array_equal(img.view(np.uint32), ref.view(np.uint32), err_msg=f"{mode} blur {blur} {params}")
        assert st.queries == q, (mode, blur, params, st.queries, q)
