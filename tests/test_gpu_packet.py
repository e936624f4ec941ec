"""The packet walk of primary rays (rt_params.packet; k_trace_split<true, .., PACKET>).

Each frame block's 64 primary rays are walked as one wave-uniform packet through the culling BVH when the block is made,
and the block hands its samples out with the first hit resolved. The (t, slot) minimum does not depend on the order
spheres are tested in, so images and query counts must equal the per-lane walk's (packet 1) and the oracle's bit for
bit. The cases aim at the packet's own rules: lanes outside the image (ragged 8x8 tiles) and uncovered rays (focal length
0 and blur 0: d = 0) take no part; tiles whose rays' direction signs disagree (a coordinate plane of the direction
crosses the tile) stay unresolved and walk per lane; bounce cap 0 makes no query; tie-heavy coincident spheres need the
lowest slot; the work-stealing and counting instantiations. The packet is opt-in (packet 2): it measured slower on C3
(DESIGN.md §4 Round 6). Box / sphere test counts differ (the packet counts its union's
tests), so a packet that silently never ran would show as equal counts.
"""
import numpy as np
import pytest

import hrt
import scenes
from hrt import Camera, Vec3, f32

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if hrt.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on an MI355X box (there is no CPU fallback)")


def _draw(sd, **params):
    r = scenes.make_renderer(sd)
    r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, **params)
    r.draw_frames(sd.frames, 1000, 10)
    return r.read_image(), r.stats()


def _axis_camera_c3(w, h, frames):
    """The cover scene seen straight along -z from x = y = 0 (height 0.3 above the ground's top): the image's middle
    column and row are the planes d.x = 0 and d.y = 0, so the tiles they cross hold rays of both signs."""
    sd = scenes.config_c3(w, h, frames)
    sd.camera = Camera.new(Vec3(0.0, 0.3, 14.0), Vec3(0.0, 0.3, 0.0), 14.0, 0.05, f32(30.0) * hrt.PI / f32(180.0))
    return sd


def _coincident(frames=2):
    base = [hrt.Sphere.new_lambertian(Vec3(0.0, 0.0, -3.0), 1.0, Vec3(0.9, 0.3, 0.2))]
    base += [hrt.Sphere.new_metal(Vec3(0.0, 0.0, -3.0), 1.0, Vec3(0.1 * k, 0.8, 0.5), 0.05 * k) for k in range(1, 8)]
    sph = np.tile(hrt.spheres_array(base), 8)  # 64 coincident spheres: every t ties, the lowest slot wins
    cam = Camera.new(Vec3(0.0, 0.5, 1.0), Vec3(0.0, 0.0, -3.0), 4.0, 0.0, 0.9)
    return scenes.SceneDef("coincident64", hrt.RT_MODE_SPHERE, 40, 27, cam, sph, frames=frames, bounces=8,
                           min_sphere_slots=0)


CASES = {
    "c3_ragged": lambda: scenes.config_c3(90, 53, 5),
    "c3_axis_planes": lambda: _axis_camera_c3(96, 64, 4),
    "coincident": _coincident,
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("steal", [1, 2])
def test_packet_equals_per_lane_walk_and_oracle(case, steal):
    sd = CASES[case]()
    img1, st1 = _draw(sd, packet=1, steal=steal, count_tests=1)
    img2, st2 = _draw(sd, packet=2, steal=steal, count_tests=1)
    assert st1.kernel.decode().endswith("false>") and st2.kernel.decode().endswith("true>"), (st1.kernel, st2.kernel)
    np.testing.assert_array_equal(img1.view(np.uint32), img2.view(np.uint32), err_msg=f"{case} steal {steal}")
    assert st1.queries == st2.queries
    assert st1.box_tests != st2.box_tests  # the packet ran (it counts its union's tests)
    ref, q = scenes.oracle_render(sd)
    np.testing.assert_array_equal(img2.view(np.uint32), ref.view(np.uint32), err_msg=f"{case} vs oracle")
    assert st2.queries == q
    img0, st0 = _draw(sd, packet=2, steal=steal, count_tests=0)  # the uncounted (timed) instantiation
    np.testing.assert_array_equal(img0.view(np.uint32), ref.view(np.uint32), err_msg=f"{case} uncounted")
    assert st0.queries == q


def test_packet_with_uncovered_rays_and_zero_bounces():
    """focal length 0 and blur 0: every primary ray has d = 0 (2a = 0: bvh_begin's uncovered rule, the exact full scan)
    and no lane takes part in the packet; bounce cap 0: no query at all (the sky colour)."""
    sd = scenes.config_c3(40, 24, 3)
    sd.camera = Camera.new(Vec3(13.0, 2.0, 3.0), Vec3(0.0, 0.0, 0.0), 0.0, 0.0, f32(20.0) * hrt.PI / f32(180.0))
    for bounces in (0, 3):
        sd.bounces = bounces
        img2, st2 = _draw(sd, packet=2)
        ref, q = scenes.oracle_render(sd)
        np.testing.assert_array_equal(img2.view(np.uint32), ref.view(np.uint32), err_msg=f"focal 0, bounces {bounces}")
        assert st2.queries == q


def test_packet_is_opt_in_and_needs_the_lds_nodes():
    """packet 0 (auto) walks every primary ray per lane (the packet measured slower on C3); packet 2 on a tree too deep
    for the LDS nodes (two cover scenes: > 192 nodes) falls back to the per-lane walk too — same bits throughout."""
    sd = scenes.config_c3(64, 40, 3)
    img, st = _draw(sd)
    assert st.kernel.decode().startswith("k_trace_split<true") and st.kernel.decode().endswith(", false>"), st.kernel
    deep = scenes.config_c3(64, 40, 3)
    deep.spheres = np.concatenate([scenes.rtiow_spheres(42), scenes.rtiow_spheres(7)])
    img_d, st_d = _draw(deep, packet=2)
    assert st_d.kernel.decode().startswith("k_trace_split<false") and st_d.kernel.decode().endswith("false>")
    for s, i, st in ((sd, img, st), (deep, img_d, st_d)):
        ref, q = scenes.oracle_render(s)
        np.testing.assert_array_equal(i.view(np.uint32), ref.view(np.uint32), err_msg=s.name)
        assert st.queries == q
