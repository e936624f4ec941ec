"""Host-side builders (product C++ in hello-raytracing_amd/csrc/host) vs the reference's unit tests and an
independent numpy restatement (oracle/host_oracle.py). CPU only."""
import math

import numpy as np
import pytest

import hrt
import scenes
from hrt import Material, Mesh, Tree, Vec3, read_asset
from oracle import host_oracle as H

LAMB = Material.new_lambertian(Vec3(0.5, 0.5, 0.5))


# ---- reference unit tests: src/geometry/mesh.rs:64-89, src/scene/bvh/tree.rs:93-126
def test_mesh_simple_cube():
    assert Mesh.load_obj(read_asset("cube.obj"), LAMB).counts() == (8, 36)


def test_mesh_suzanne():
    assert Mesh.load_obj(read_asset("suzanne.obj"), LAMB).counts() == (515, 2937)


def test_tree_simple_cube():
    t = Tree.from_mesh(Mesh.load_obj(read_asset("cube.obj"), LAMB))
    t.build()
    sizes, nodes, tris, mats = t.view()
    assert sizes == [16, 12] and len(nodes) == 16 and len(tris) == 12 and len(mats) == 1


def test_tree_suzanne():
    t = Tree.from_mesh(Mesh.load_obj(read_asset("suzanne.obj"), LAMB))
    t.build()
    sizes, nodes, tris, mats = t.view()
    assert sizes == [1024, 979] and len(nodes) == 1024 and len(tris) == 979 and len(mats) == 1


# ---- byte-for-byte against the numpy restatement
@pytest.mark.parametrize("args", [
    ((0.0, 0.0, 3.5), (0.0, 0.0, 0.0), 3.5, 0.04, float(np.float32(math.pi) * np.float32(0.2))),
    ((3.0, 1.5, -2.0), (0.0, 0.0, -5.0), 5.0, 0.1, 0.8),
    ((13.0, 2.0, 3.0), (0.0, 0.0, 0.0), 10.0, 0.05, 0.3490658),
    ((0.0, 2.2, 4.5), (0.0, 0.0, -4.5), 5.6, 0.0, float(np.float32(math.pi) * np.float32(0.3))),
])
def test_camera_new_matches_glam_restatement(args):
    frm, to, focal, blur, fov = args
    got = hrt.Camera.new(Vec3(*frm), Vec3(*to), focal, blur, fov)
    want = H.camera_new(frm, to, np.float32(focal), np.float32(blur), np.float32(fov))
    assert np.frombuffer(got.tobytes(), dtype=np.uint32).tolist() == want.view(np.uint32).tolist()


def _tree_bytes_match(asset_mats):
    t = Tree()
    meshes = []
    for k, (name, mat) in enumerate(asset_mats):
        raw = read_asset(name)
        t.add_mesh(Mesh.load_obj(raw, mat))
        corners, _ = H.parse_obj(raw.decode())
        meshes.append(([c for m in corners for c in m], k))
    t.build()
    sizes, nodes, tris, _ = t.view()
    wsizes, wnodes, wtris = H.tree_build(meshes)
    assert sizes == wsizes
    assert nodes.view(np.uint32).reshape(-1).tolist() == wnodes.view(np.uint32).reshape(-1).tolist()
    for got, want in zip(tris, wtris):
        for field, w in zip(("a", "b", "c", "custom"), want[:4]):
            assert got[field].view(np.uint32).tolist() == np.asarray(w, np.float32).view(np.uint32).tolist()
        assert got["material"] == want[4]


def test_tree_build_suzanne_matches_restatement():
    _tree_bytes_match([("suzanne.obj", LAMB)])


def test_tree_build_new_suzane_scene_matches_restatement():
    """The five-mesh tree of SceneTris::new_suzane (scene_tris.rs:119-145): 1095 triangles, n = 2048."""
    _tree_bytes_match([("suzanne.obj", LAMB), ("ico_sphere.obj", Material.new_dielectric(0.2)),
                       ("cube_s.obj", LAMB), ("cube_m.obj", LAMB), ("cube_l.obj", LAMB)])
    assert hrt.SceneTris.build_suzane_tree().sizes == [2048, 1095]


def test_tree_build_lucy_matches_restatement():
    _tree_bytes_match([("lucy_lp_20.obj", LAMB), ("floor.obj", LAMB)])


def test_parallel_tree_build_is_byte_identical():
    """the level-synchronous multi-threaded Tree::build equals the sequential one byte for
    byte (dragon: 49,988 triangles, n = 65536; lucy) for several thread counts."""
    for asset in ("xyzrgb_dragon_lp_20.obj", "lucy_lp_20.obj"):
        views = []
        for threads in (1, 3, 8, 16):
            t = Tree.from_mesh(Mesh.load_obj(hrt.read_asset(asset), LAMB))
            t.add_mesh(Mesh.load_obj(hrt.read_asset("floor.obj"), LAMB))
            t.build(threads=threads)
            sizes, nodes, tris, mats = t.view()
            views.append((sizes, nodes.tobytes(), tris.tobytes(), mats.tobytes()))
        assert all(v == views[0] for v in views[1:]), asset
    assert views[0][0] == [32768, 19929]  # lucy


# ---- OBJ edge cases (tobj behaviour the reference relies on)
def test_obj_negative_indices_models_and_quads():
    src = b"""o A
v 0 0 0
v 1 0 0
v 0 1 0
v 1 1 0
f -4 -3 -2
g B
f 2/7/1 4//2 3
f 1 2 4 3
"""
    m = Mesh.load_obj(src, LAMB)
    # model A: 3 unique positions, model B: 4 unique; quad kept as 4 corners (triangulate = false)
    assert m.counts() == (7, 3 + 3 + 4)
    t = Tree.from_mesh(m)
    t.build()
    sizes, _, tris, _ = t.view()
    assert sizes == [4, 3]  # 10 corners -> chunks_exact(3) -> 3 triangles


@pytest.mark.parametrize("bad", [b"v 0 0\nf 1 1 1\n", b"v 0 0 zero\n", b"v 0 0 0\nf 1 2 3\n", b"v 0 0 0\nf 0 1 1\n"])
def test_obj_load_error_gives_empty_mesh(bad):
    assert Mesh.load_obj(bad, LAMB).counts() == (0, 0)


def test_empty_tree_build():
    t = Tree()
    t.build()
    assert t.sizes == [1, 0]


# ---- render_ppm / compare_ppm_images (render_ppm.rs:38-57, rendering_tests.rs:84-131)
def test_render_ppm_format_and_saturating_cast():
    img = np.array([[[0.0, 1.0, 0.5], [-1.0, 2.0, np.nan]], [[0.999, 1e-9, 255.0], [0.00392, 0.1, 0.2]]],
                   dtype=np.float32)
    ppm = hrt.ppm_from_image(img, 2, 2)
    assert ppm == "P3\n2 2 255\n0 255 127 0 255 0 254 0 255 0 25 51 "
    assert np.array_equal(scenes.to_u8(img).reshape(-1), [0, 255, 127, 0, 255, 0, 254, 0, 255, 0, 25, 51])


def test_compare_ppm_images_semantics():
    a = scenes.ppm_text_from_u8(np.full((4, 4, 3), 100, np.uint8))
    b = scenes.ppm_text_from_u8(np.full((4, 4, 3), 104, np.uint8))  # 4/255 = 1.57 %
    assert abs(hrt.compare_ppm_images(a, b, 2.0) - 4 / 255 * 100) < 1e-4
    with pytest.raises(hrt.ComparisonError) as e:
        hrt.compare_ppm_images(a, b, 1.0)
    assert e.value.kind == "ExcessiveDifference"
    c = scenes.ppm_text_from_u8(np.full((4, 5, 3), 100, np.uint8))
    with pytest.raises(hrt.ComparisonError) as e:
        hrt.compare_ppm_images(a, c, 2.0)
    assert e.value.kind == "DifferentDimensions"
    with pytest.raises(hrt.ComparisonError) as e:
        hrt.compare_ppm_images(a, a + "7 ", 2.0)
    assert e.value.kind == "PixelCountMismatch"


def test_rtiow_scene_is_deterministic():
    a, b = scenes.rtiow_spheres(), scenes.rtiow_spheres()
    assert a.tobytes() == b.tobytes() and 450 <= len(a) <= 500
