"""Scene definitions shared by the tests, bench.py and smoke().

golden_scene(name) restates the seven scene builders of the reference's golden harness
(tests/rendering_tests.rs:134-509) with the hrt host API. config_*() define the synthetic benchmark
workloads of BASELINE.json (the reference cannot express them): C1 single sphere, C2 three
spheres, C3 RTIOW-style cover scene (seeded), C4 Suzanne + ground sphere (mixed mode).
"""
from __future__ import annotations

import gzip
import json
import math
from dataclasses import dataclass
from pathlib import Path

import numpy as np

import hrt
from hrt import PI, Camera, Sphere, Vec3, f32

GOLDEN_DIR = Path(__file__).resolve().parent / "golden"
GOLDEN_FRAMES = 100  # goldens were produced with 100 frames, time 1000 + 10 i
GOLDEN_NAMES = ["lambertian_materials", "metal_materials", "dielectric_materials", "camera_position",
                "depth_of_field", "complex_scene", "shadow_rendering"]
GLASS_GOLDENS = {"dielectric_materials", "complex_scene"}


@dataclass
class SceneDef:
    name: str
    mode: int
    width: int
    height: int
    camera: np.ndarray
    spheres: np.ndarray | None = None
    bvh: tuple | None = None
    frames: int = 100
    bounces: int | None = None
    min_sphere_slots: int | None = None


def default_sphere_camera() -> np.ndarray:
    # SceneSphere::new, scene_sphere.rs:38-39
    return Camera.new(Vec3(0.0, 0.0, 3.5), Vec3(0.0, 0.0, 0.0), 3.5, 0.04, PI * f32(0.2))


def golden_scene(name: str, width: int = 512, height: int = 512) -> SceneDef:
    cam = default_sphere_camera()
    o = []
    if name == "lambertian_materials":  # rendering_tests.rs:134-170
        o += [Sphere.new_lambertian(Vec3(-2.0, 0.0, -5.0), 1.0, Vec3(0.8, 0.2, 0.2)),
              Sphere.new_lambertian(Vec3(0.0, 0.0, -5.0), 1.0, Vec3(0.2, 0.8, 0.2)),
              Sphere.new_lambertian(Vec3(2.0, 0.0, -5.0), 1.0, Vec3(0.2, 0.2, 0.8)),
              Sphere.new_lambertian(Vec3(0.0, -101.0, -5.0), 100.0, Vec3(0.5, 0.5, 0.5))]
    elif name == "metal_materials":  # :188-227
        o += [Sphere.new_metal(Vec3(-2.0, 0.0, -5.0), 1.0, Vec3(0.8, 0.8, 0.8), 0.0),
              Sphere.new_metal(Vec3(0.0, 0.0, -5.0), 1.0, Vec3(0.8, 0.6, 0.2), 0.2),
              Sphere.new_metal(Vec3(2.0, 0.0, -5.0), 1.0, Vec3(0.6, 0.2, 0.8), 0.5),
              Sphere.new_lambertian(Vec3(0.0, -101.0, -5.0), 100.0, Vec3(0.5, 0.5, 0.5))]
    elif name == "dielectric_materials":  # :245-287
        o += [Sphere.new_dielectric(Vec3(0.0, 0.0, -5.0), 1.5, 1.5),
              Sphere.new_dielectric(Vec3(-2.0, 0.0, -4.0), 0.5, 1.33),
              Sphere.new_dielectric(Vec3(2.0, 0.0, -4.0), 0.5, 2.4),
              Sphere.new_lambertian(Vec3(0.0, 0.0, -8.0), 1.0, Vec3(1.0, 0.0, 0.0)),
              Sphere.new_lambertian(Vec3(0.0, -101.5, -5.0), 100.0, Vec3(0.5, 0.5, 0.5))]
    elif name == "camera_position":  # :305-338
        for i in range(-2, 3):
            o.append(Sphere.new_lambertian(Vec3(f32(i) * f32(1.5), 0.0, f32(-5.0) - f32(abs(i))), 0.5,
                                           Vec3(f32(0.5) + f32(i) * f32(0.1), 0.5, f32(0.5) - f32(i) * f32(0.1))))
        o.append(Sphere.new_lambertian(Vec3(0.0, -100.5, -5.0), 100.0, Vec3(0.5, 0.5, 0.5)))
        cam = Camera.new(Vec3(3.0, 1.5, -2.0), Vec3(0.0, 0.0, -5.0), 5.0, 0.1, 0.8)
    elif name == "depth_of_field":  # :356-394
        for i in range(-3, 4):
            z = f32(-3.0) - f32(abs(i)) * f32(2.0)
            o.append(Sphere.new_lambertian(Vec3(f32(i), 0.0, z), 0.4,
                                           Vec3(f32(1.0) - f32(i + 3) / f32(6.0), 0.5, f32(i + 3) / f32(6.0))))
        o.append(Sphere.new_lambertian(Vec3(0.0, -100.4, -5.0), 100.0, Vec3(0.5, 0.5, 0.5)))
        cam = Camera.new(Vec3(0.0, 1.0, 0.0), Vec3(0.0, 0.0, -5.0), 5.0, 0.3, 0.8)
    elif name == "complex_scene":  # :412-462
        for i in range(-2, 3):
            for j in range(-2, 3):
                if i == 0 and j == 0:
                    o.append(Sphere.new_dielectric(Vec3(0.0, 0.0, -5.0), 0.8, 1.5))
                    continue
                x = f32(i) * f32(1.2)
                z = f32(-5.0) + f32(j) * f32(1.2)
                kind = abs(i + j) % 3
                if kind == 0:
                    o.append(Sphere.new_lambertian(Vec3(x, 0.0, z), 0.3, Vec3(0.7, 0.3, 0.3)))
                elif kind == 1:
                    o.append(Sphere.new_metal(Vec3(x, 0.0, z), 0.3, Vec3(0.7, 0.7, 0.7), 0.1))
                else:
                    o.append(Sphere.new_dielectric(Vec3(x, 0.0, z), 0.3, 1.33))
        o.append(Sphere.new_lambertian(Vec3(0.0, -100.3, -5.0), 100.0, Vec3(0.5, 0.5, 0.5)))
    elif name == "shadow_rendering":  # :480-509
        o += [Sphere.new_lambertian(Vec3(0.0, 2.0, -5.0), 2.0, Vec3(0.7, 0.3, 0.3)),
              Sphere.new_lambertian(Vec3(0.0, -0.5, -5.0), 0.5, Vec3(0.3, 0.7, 0.3)),
              Sphere.new_lambertian(Vec3(0.0, -101.0, -5.0), 100.0, Vec3(0.8, 0.8, 0.8))]
    elif name == "performance":  # :527-557 (21 spheres)
        for i in range(20):
            angle = f32(i) * f32(math.pi) * f32(2.0) / f32(20.0)
            x = f32(np.cos(angle)) * f32(3.0)
            z = f32(-5.0) + f32(np.sin(angle)) * f32(3.0)
            o.append(Sphere.new_lambertian(Vec3(x, 0.0, z), 0.4,
                                           Vec3(f32(i) / f32(20.0), 0.5, f32(1.0) - f32(i) / f32(20.0))))
        o.append(Sphere.new_lambertian(Vec3(0.0, -100.4, -5.0), 100.0, Vec3(0.5, 0.5, 0.5)))
    else:
        raise KeyError(name)
    return SceneDef(name, hrt.RT_MODE_SPHERE, width, height, cam, hrt.spheres_array(o), frames=GOLDEN_FRAMES)


def load_golden_u8(name: str) -> np.ndarray:
    """Reference golden image as u8 [H, W, 3] (tests/golden/ppm/, converted by make_fixtures.py)."""
    man = json.loads((GOLDEN_DIR / "ppm/manifest.json").read_text())[name]
    raw = gzip.decompress((GOLDEN_DIR / f"ppm/{name}.u8.gz").read_bytes())
    return np.frombuffer(raw, dtype=np.uint8).reshape(man["height"], man["width"], 3)


def ppm_text_from_u8(u8: np.ndarray) -> str:
    """ASCII P3 text of a u8 image in render_ppm's exact format (render_ppm.rs:51-55)."""
    h, w, _ = u8.shape
    return f"P3\n{w} {h} 255\n" + "".join(f"{v} " for v in u8.reshape(-1).tolist())


def to_u8(img: np.ndarray) -> np.ndarray:
    """render_ppm's `(v * 255.0) as u8` (render_ppm.rs:48-49): f32 multiply, saturate, truncate, NaN -> 0."""
    v = np.asarray(img, dtype=np.float32) * np.float32(255.0)
    v = np.where(np.isnan(v), np.float32(0.0), v)
    return np.clip(np.trunc(v), 0, 255).astype(np.uint8)


# ------------------------------------------------------------------------------------- benchmark configs
def _pcg_stream(seed: int):
    """Deterministic u32 stream (the shaders' PCG hash step) for the seeded scene generators."""
    s = seed & 0xFFFFFFFF
    while True:
        old = (s + 747796405 + 2891336453) & 0xFFFFFFFF
        word = (((old >> ((old >> 28) + 4)) ^ old) * 277803737) & 0xFFFFFFFF
        s = ((word >> 22) ^ word) & 0xFFFFFFFF
        yield s


def config_c1() -> SceneDef:
    """C1: single Lambertian sphere, 400x225, 16 spp, 8 bounces (camera of new_simple, scene_sphere.rs:96-102)."""
    cam = Camera.new(Vec3(0.0, 0.2, 1.5), Vec3(0.0, 0.1, -3.0), 2.2, 0.05, PI * f32(0.3))
    sp = hrt.spheres_array([Sphere.new_lambertian(Vec3(0.0, 0.0, -1.0), 0.5, Vec3(0.5, 0.5, 0.5))])
    return SceneDef("C1-single-sphere", hrt.RT_MODE_SPHERE, 400, 225, cam, sp, frames=16, bounces=8,
                    min_sphere_slots=0)


def config_c2(width: int = 1280, height: int = 720, frames: int = 256) -> SceneDef:
    """C2: ground + Lambertian / Metal(0.1) / Dielectric(1.5), 1280x720, 256 spp, 50 bounces."""
    cam = Camera.new(Vec3(0.0, 0.2, 1.5), Vec3(0.0, 0.1, -3.0), 2.2, 0.05, PI * f32(0.3))
    sp = hrt.spheres_array([
        Sphere.new_lambertian(Vec3(0.0, -100.5, -1.0), 100.0, Vec3(0.12, 0.12, 0.18)),
        Sphere.new_lambertian(Vec3(0.0, 0.0, -1.0), 0.5, Vec3(0.1, 0.2, 0.5)),
        Sphere.new_metal(Vec3(1.0, 0.0, -1.0), 0.5, Vec3(0.8, 0.6, 0.2), 0.1),
        Sphere.new_dielectric(Vec3(-1.0, 0.0, -1.0), 0.5, 1.5),
    ])
    return SceneDef("C2-three-spheres", hrt.RT_MODE_SPHERE, width, height, cam, sp, frames=frames, bounces=50,
                    min_sphere_slots=0)


def rtiow_spheres(seed: int = 42) -> np.ndarray:
    """RTIOW 'final scene' layout (public book, not the reference): ground r=1000, 22x22 jittered small
    spheres (~80 % Lambertian, 15 % metal, 5 % glass) skipping those near (4, 0.2, 0), 3 big spheres.
    Seeded and deterministic (PCG stream), ~488 spheres."""
    g = _pcg_stream(seed)

    def rnd() -> np.float32:
        return np.float32(next(g)) * np.float32(2.0 ** -32)

    o = [Sphere.new_lambertian(Vec3(0.0, -1000.0, 0.0), 1000.0, Vec3(0.5, 0.5, 0.5))]
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = rnd()
            cx = f32(a) + f32(0.9) * rnd()
            cz = f32(b) + f32(0.9) * rnd()
            if (cx - 4.0) ** 2 + (0.2 - 0.2) ** 2 + cz ** 2 <= 0.81:
                continue
            c = Vec3(cx, 0.2, cz)
            if choose < 0.8:
                alb = Vec3(rnd() * rnd(), rnd() * rnd(), rnd() * rnd())
                o.append(Sphere.new_lambertian(c, 0.2, alb))
            elif choose < 0.95:
                alb = Vec3(f32(0.5) + f32(0.5) * rnd(), f32(0.5) + f32(0.5) * rnd(), f32(0.5) + f32(0.5) * rnd())
                o.append(Sphere.new_metal(c, 0.2, alb, f32(0.5) * rnd()))
            else:
                o.append(Sphere.new_dielectric(c, 0.2, 1.5))
    o.append(Sphere.new_dielectric(Vec3(0.0, 1.0, 0.0), 1.0, 1.5))
    o.append(Sphere.new_lambertian(Vec3(-4.0, 1.0, 0.0), 1.0, Vec3(0.4, 0.2, 0.1)))
    o.append(Sphere.new_metal(Vec3(4.0, 1.0, 0.0), 1.0, Vec3(0.7, 0.6, 0.5), 0.0))
    return hrt.spheres_array(o)


def rtiow_camera() -> np.ndarray:
    # lookfrom (13,2,3) -> lookat (0,0,0), focus distance 10, defocus ~0.05, vfov 20 degrees
    return Camera.new(Vec3(13.0, 2.0, 3.0), Vec3(0.0, 0.0, 0.0), 10.0, 0.05, f32(20.0) * PI / f32(180.0))


def config_c3(width: int = 1920, height: int = 1080, frames: int = 1024) -> SceneDef:
    """C3 (the headline metric): RTIOW cover scene, 1920x1080, 1024 spp, 50 bounces."""
    return SceneDef("C3-rtiow-cover", hrt.RT_MODE_SPHERE, width, height, rtiow_camera(), rtiow_spheres(),
                    frames=frames, bounces=50, min_sphere_slots=0)


def suzanne_tree() -> "hrt.Tree":
    from hrt import Material, Mesh, Tree, read_asset
    t = Tree.from_mesh(Mesh.load_obj(read_asset("suzanne.obj"), Material.new_lambertian(Vec3(0.3, 0.4, 0.6))))
    t.build()
    return t


def config_c4(width: int = 1920, height: int = 1080, frames: int = 512) -> SceneDef:
    """C4: suzanne.obj (979 triangles, BVH n=1024) + a ground sphere, mixed mode, camera of new_suzane."""
    bvh = suzanne_tree().view()
    ground = hrt.spheres_array([Sphere.new_lambertian(Vec3(0.0, -101.0, -4.5), 100.0, Vec3(0.5, 0.5, 0.6))])
    cam = Camera.new(Vec3(0.0, 2.2, 4.5), Vec3(0.0, 0.0, -4.5), 5.6, 0.0, PI * f32(0.3))
    return SceneDef("C4-suzanne-ground", hrt.RT_MODE_MIXED, width, height, cam, ground, bvh=bvh, frames=frames,
                    bounces=50, min_sphere_slots=0)


def config_c5(width: int = 3840, height: int = 2160, frames: int = 4096) -> SceneDef:
    """C5: the C3 cover scene plus suzanne.obj (979 triangles, mesh at its file coordinates), mixed mode,
    3840x2160, 4096 spp, 50 bounces (BASELINE: row tiles across 8 GPUs)."""
    bvh = suzanne_tree().view()
    return SceneDef("C5-rtiow-suzanne-4k", hrt.RT_MODE_MIXED, width, height, rtiow_camera(), rtiow_spheres(),
                    bvh=bvh, frames=frames, bounces=50, min_sphere_slots=0)


CONFIGS = {"c1": config_c1, "c2": config_c2, "c3": config_c3, "c4": config_c4, "c5": config_c5}


def make_renderer(sd: SceneDef) -> "hrt.Renderer":
    """GPU renderer loaded with a SceneDef (camera, buffers, params)."""
    r = hrt.Renderer(sd.width, sd.height, sd.mode)
    kw = {"count_tests": 1}  # (the tests compare work counts; bench.py turns the counting off for its timed steps)
    if sd.bounces is not None:
        kw["bounces"] = sd.bounces
    if sd.min_sphere_slots is not None:
        kw["min_sphere_slots"] = sd.min_sphere_slots
    r.set_params(**kw)
    r.set_camera(sd.camera)
    if sd.mode != hrt.RT_MODE_TRIS:
        r.write_spheres(sd.spheres if sd.spheres is not None else hrt.spheres_array([]))
    if sd.mode != hrt.RT_MODE_SPHERE and sd.bvh is not None:
        r.write_bvh(*sd.bvh)
    return r


def oracle_render(sd: SceneDef, **kw):
    """The CPU oracle on a SceneDef (tests / cpu_baseline only)."""
    from oracle import oracle as O
    args = dict(width=sd.width, height=sd.height, mode=sd.mode, camera=sd.camera, frames=sd.frames,
                spheres=sd.spheres, bvh=sd.bvh, bounces=sd.bounces, min_sphere_slots=sd.min_sphere_slots)
    args.update(kw)
    return O.render(**args)


# ---- committed oracle fixtures (tests/golden/oracle, made by tests/golden/make_oracle_fixtures.py)
ORACLE_FIXTURE_DIR = GOLDEN_DIR / "oracle"


def _tris_scene(name: str, width: int, height: int, frames: int) -> SceneDef:
    from hrt import SceneTris
    if name == "suzane":
        tree, cam = SceneTris.build_suzane_tree(), SceneTris.suzane_camera()
    else:  # dragon on the floor (scene_tris.rs:67-92): its walks hit the 600-step cap
        tree = SceneTris._mesh_on_floor("xyzrgb_dragon_lp_20.obj", Vec3(0.7, 0.7, 0.2))
        cam = Camera.new(Vec3(0.0, 2.0, 8.0), Vec3(0.0, 0.0, -8.0), 5.6, 0.0, PI * f32(0.3))
    return SceneDef(name, hrt.RT_MODE_TRIS, width, height, cam, bvh=tree.view(), frames=frames)


def oracle_fixture_cases():
    """name -> (SceneDef, (row0, row_step)): full-width row subsets (rows row0, row0 + step, ... to the
    bottom, the set a renderer with rt_params.row0/row_step draws) of every BASELINE config and of the
    golden and triangle scenes, few frames each."""
    def frames(sd, f):
        sd.frames = f
        return sd
    return {
        "golden_complex_scene_64": (frames(golden_scene("complex_scene", 64, 64), 10), (0, 1)),
        "golden_dielectric_64": (frames(golden_scene("dielectric_materials", 64, 64), 10), (0, 1)),
        "c1": (config_c1(), (2, 15)),
        "c2": (frames(config_c2(), 2), (7, 90)),
        "c3": (frames(config_c3(), 2), (13, 180)),
        "c4": (frames(config_c4(), 2), (17, 180)),
        "c5": (frames(config_c5(), 1), (29, 540)),
        "tris_suzane": (_tris_scene("suzane", 160, 120, 3), (1, 4)),
        "tris_dragon": (_tris_scene("dragon", 96, 72, 2), (0, 3)),
    }


def oracle_fixture_trees():
    """name -> Tree (host builders) whose bytes are pinned by tests/golden/oracle/trees.json."""
    from hrt import Material, Mesh, SceneTris, Tree, read_asset
    lamb = Material.new_lambertian(Vec3(0.5, 0.5, 0.5))

    def one(asset):
        t = Tree.from_mesh(Mesh.load_obj(read_asset(asset), lamb))
        t.build()
        return t
    return {
        "cube": lambda: one("cube.obj"),
        "suzanne": lambda: one("suzanne.obj"),
        "new_suzane": SceneTris.build_suzane_tree,
        "dragon_floor": lambda: SceneTris._mesh_on_floor("xyzrgb_dragon_lp_20.obj", Vec3(0.7, 0.7, 0.2)),
        "lucy_floor": lambda: SceneTris._mesh_on_floor("lucy_lp_20.obj", Vec3(0.4, 0.3, 0.6)),
    }


def tree_digest(tree) -> dict:
    import hashlib
    sizes, nodes, tris, mats = tree.view()
    return {"sizes": list(sizes), "nodes_sha256": hashlib.sha256(nodes.tobytes()).hexdigest(),
            "tris_sha256": hashlib.sha256(tris.tobytes()).hexdigest(),
            "mats_sha256": hashlib.sha256(mats.tobytes()).hexdigest()}


def load_oracle_fixture(name: str):
    """(image float32 [rows, W, 3], manifest entry) of a committed oracle fixture."""
    man = json.loads((ORACLE_FIXTURE_DIR / "manifest.json").read_text())[name]
    with np.load(ORACLE_FIXTURE_DIR / "images.npz", allow_pickle=False) as z:
        img = z[name].copy()
    return img, man

