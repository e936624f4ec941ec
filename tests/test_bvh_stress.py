"""Stress tests of the culling sphere BVH's exactness (variant 4; DESIGN.md §4 "Sphere BVH exactness").

The culling BVH may only skip a sphere the reference's float arithmetic would reject. Its boxes are padded by
2.02 delta, delta a bound on how far outside a sphere a ray can pass while the reference's f32 discriminant
(shader_sphere.wgsl:136-155) still reports a hit. Two checks:

* GPU (`-m gpu`): fixed-seed adversarial scenes — radius ratios of 1e6, coincident and concentric spheres,
  tight clusters, a grazing camera along a tangent row — rendered with the exact linear scan (variant 1) and
  the culling BVH (variant 4) under both schedules (tiles: k_render; sample queue: k_trace_split, nodes in
  LDS or not): bit-identical images and identical closest-hit query counts over more than 1e8 rays.
* CPU: the margin itself. For random rays, including rays built to graze each sphere, the f32 discriminant is
  evaluated exactly as the kernels do (fma emulated in float64) and, for every sphere it accepts, the true
  distance h from the centre to the ray line is compared with the radius: the worst (h - r) / delta over all
  accepted pairs must stay below 1 (the padding leaves a factor of 2.02).
"""
import math

import numpy as np
import pytest

import hrt
import scenes

U = 2.0 ** -24


def stress_scene(kind: str, seed: int = 11, width: int = 640, height: int = 480, frames: int = 64):
    rng = np.random.default_rng(seed)
    o = []
    mats = [lambda c, r: hrt.Sphere.new_lambertian(c, r, hrt.Vec3(*rng.uniform(0.1, 0.9, 3))),
            lambda c, r: hrt.Sphere.new_metal(c, r, hrt.Vec3(*rng.uniform(0.3, 0.9, 3)), float(rng.uniform(0, 0.4))),
            lambda c, r: hrt.Sphere.new_dielectric(c, r, float(rng.choice([1.33, 1.5, 2.4])))]
    cam_from, cam_to, fov = (0.5, 2.0, 3.0), (0.0, 0.0, -5.0), 0.9
    if kind == "radius_1e6":  # radii over six decades, small spheres next to huge ones
        for _ in range(300):
            c = rng.uniform([-6, -2, -14], [6, 4, -2])
            o.append(mats[rng.integers(3)](hrt.Vec3(*c), float(10 ** rng.uniform(-3, 3) * 1e-3)))
        for _ in range(6):
            c = rng.uniform([-6, -2, -14], [6, 4, -2])
            o.append(mats[rng.integers(3)](hrt.Vec3(*c), float(10 ** rng.uniform(-1, 0.3))))
    elif kind == "coincident":  # exact duplicates (slot ties) and concentric shells
        for _ in range(40):
            c = rng.uniform([-4, -1, -9], [4, 3, -2])
            r = float(rng.uniform(0.05, 0.6))
            for _ in range(int(rng.integers(1, 4))):
                o.append(mats[rng.integers(3)](hrt.Vec3(*c), r))
            o.append(mats[rng.integers(3)](hrt.Vec3(*c), r * float(rng.uniform(0.3, 0.99))))
    elif kind == "clustered":  # clusters of near-identical spheres 1e-4 apart
        for _ in range(12):
            c0 = rng.uniform([-4, -1, -9], [4, 3, -2])
            r0 = float(rng.uniform(0.1, 0.5))
            for _ in range(24):
                c = c0 + rng.uniform(-1e-4, 1e-4, 3)
                o.append(mats[rng.integers(3)](hrt.Vec3(*c), r0 * float(1.0 + rng.uniform(-1e-4, 1e-4))))
    elif kind == "grazing":  # a row of spheres tangent to one plane, the camera sliding along that plane
        for i in range(-30, 30):
            r = 0.25 * (1.0 + 0.5 * math.sin(i))
            o.append(mats[i % 3](hrt.Vec3(0.3 * i, r, -6.0 - 0.01 * i), r))
            o.append(mats[(i + 1) % 3](hrt.Vec3(0.3 * i + 0.15, -r, -6.5), r))
        cam_from, cam_to, fov = (-12.0, 0.0, -6.2), (12.0, 0.0, -6.2), 0.3
    else:
        raise ValueError(kind)
    o.append(hrt.Sphere.new_lambertian(hrt.Vec3(0.0, -1000.5, -5.0), 1000.0, hrt.Vec3(0.5, 0.5, 0.5)))
    cam = hrt.Camera.new(hrt.Vec3(*cam_from), hrt.Vec3(*cam_to), 6.0, 0.1, fov)
    return scenes.SceneDef(kind, hrt.RT_MODE_SPHERE, width, height, cam, hrt.spheres_array(o), frames=frames,
                           bounces=50, min_sphere_slots=0)


KINDS = ["radius_1e6", "coincident", "clustered", "grazing"]


@pytest.mark.gpu
def test_culling_bvh_stress_bit_identical():
    if hrt.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on an MI355X box (there is no CPU fallback)")
    total = 0
    kernels = set()
    for kind in KINDS:
        sd = stress_scene(kind)
        out = {}
        for variant, schedule in ((1, 2), (4, 2), (4, 1)):
            r = scenes.make_renderer(sd)
            r.set_params(variant=variant, schedule=schedule)
            r.draw_frames(sd.frames, 1000, 10)
            st = r.stats()
            out[(variant, schedule)] = (r.read_image(), st.queries, st.kernel.decode())
            r.close()
        ref_img, ref_q, _ = out[(1, 2)]
        for key in ((4, 2), (4, 1)):
            img, q, k = out[key]
            np.testing.assert_array_equal(ref_img.view(np.uint32), img.view(np.uint32), err_msg=f"{kind} {key}")
            assert q == ref_q, (kind, key, q, ref_q)
            kernels.add(k)
        total += ref_q
    assert total > 1e8, total
    # both node placements of the sample-queue kernel ran (nodes in LDS / fp16 nodes from L1/L2), whichever the
    # work-stealing instantiation (k_trace_split<LNODES, STEAL>)
    assert {k.split(",")[0] for k in kernels if k.startswith("k_trace_split<")} >= {"k_trace_split<true", "k_trace_split<false"}, kernels


def _f32(x):
    return np.asarray(x, dtype=np.float32)


def _fma32(a, b, c):
    """f32 fma emulated in float64 (the f32 x f32 product is exact in float64)."""
    return _f32(np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64))


def _accepts(o, d, c, rr):
    """The kernels' (and the reference's) f32 test: disc >= 0 and b <= 0 (exact_t_geo)."""
    oc = _f32(o - c)
    bd = _fma32(oc[..., 2], d[..., 2], _fma32(oc[..., 1], d[..., 1], _f32(oc[..., 0] * d[..., 0])))
    b = _f32(bd + bd)
    cc = _f32(_fma32(oc[..., 2], oc[..., 2], _fma32(oc[..., 1], oc[..., 1], _f32(oc[..., 0] * oc[..., 0]))) - rr)
    a = _fma32(d[..., 2], d[..., 2], _fma32(d[..., 1], d[..., 1], _f32(d[..., 0] * d[..., 0])))
    disc = _fma32(b, b, _f32(-_f32(4.0 * a) * cc))
    return (disc >= 0) & (b <= 0)


@pytest.mark.parametrize("kind", KINDS)
def test_culling_bvh_padding_margin(kind):
    sd = stress_scene(kind)
    sp = sd.spheres
    C = sp["center"].astype(np.float32)
    R = sp["radius"].astype(np.float32)
    # spheres far larger than the median (the ground) are scanned for every ray, not culled
    # (host/sphere_bvh.cpp): the BVH's delta uses the radii of the others
    inside = R <= 32.0 * np.median(R)
    C, R = C[inside], R[inside]
    rng = np.random.default_rng(5)
    n = 400_000
    k = rng.integers(len(R), size=n)
    c, r = C[k], R[k]
    # rays built to graze sphere k: origin at distance s along a random direction, aimed at a point just
    # off the silhouette (within a few ulps of tangency), plus fully random rays
    dist = (10.0 ** rng.uniform(-1, 3, n)) * np.maximum(r, 1e-3)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    o = _f32(c + u * dist[:, None])
    w = rng.normal(size=(n, 3))
    w -= (w * u).sum(1, keepdims=True) * u
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    # aim within a few float errors of tangency (the f32 test's error is ~u |w|): accepted misses live there
    eps = rng.uniform(-16.0, 16.0, n) * U * (dist + r)
    tangent = c + w * (r + eps)[:, None]
    d = _f32(tangent - o)
    scale = (10.0 ** rng.integers(-3, 4, n)).astype(np.float32)
    d = _f32(d * scale[:, None])
    acc = _accepts(o, d, c, _f32(r * r))
    od, dd, cd = o.astype(np.float64), d.astype(np.float64), c.astype(np.float64)
    wv = od - cd
    dn = np.linalg.norm(dd, axis=1)
    h = np.linalg.norm(np.cross(wv, dd), axis=1) / dn  # distance from the centre to the ray line
    excess = h - r.astype(np.float64)
    # the kernel's delta (renderer.cpp pad_k*, rt_kernels.hip bvh_begin) with D >= |w|
    rmax, rmin = float(R.max()), float(max(R[R > 0].min(), 0.0))
    D = np.linalg.norm(wv, axis=1) * 1.001
    delta = 8 * U * rmax + np.minimum(16 * U * D * D / rmin, 2e-3 * D) + 4 * U * D + 4e-23 / dn
    ratio = np.where(acc & (excess > 0), excess / delta, 0.0)
    worst = float(ratio.max())
    print(f"{kind}: {int(acc.sum())} accepted of {n} grazing pairs, worst (h - r) / delta = {worst:.3e}")
    assert acc.sum() > n // 10  # the rays do graze: many pairs are accepted
    assert worst < 1.0, worst
