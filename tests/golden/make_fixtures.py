"""Generate the committed test fixtures from the reference checkout (run once, in the build container).

Reads (read-only) /root/reference and writes:
  tests/golden/ppm/<name>.u8.gz        the reference's golden images (tests/golden/*.ppm, ASCII P3 512x512)
                                       as raw u8 RGB, row-major — data only, header checked here
  tests/golden/ppm/manifest.json       name -> {width, height, md5 of the original .ppm}
  hello-raytracing_amd/assets/*.obj.gz the OBJ meshes the reference's scenes load (src/assets)

Nothing at test or bench time reads /root/reference; the GPU box never sees it.
Duplicate goldens (camera.ppm == camera_position.ppm, complex.ppm == complex_scene.ppm) are stored once;
materials.ppm has no generator in the reference's tests and is kept only as an unpinned image.
"""
from __future__ import annotations

import gzip
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
REPO = Path(__file__).resolve().parents[2]
GOLDENS = ["lambertian_materials", "metal_materials", "dielectric_materials", "camera_position",
           "depth_of_field", "complex_scene", "shadow_rendering", "materials"]
ASSETS = ["suzanne", "suzanne_lp", "ico_sphere", "cube", "cube2", "cube_s", "cube_m", "cube_l", "floor", "quad",
          "lucy_lp_20"]


def parse_p3(text: str):
    lines = text.split("\n")
    assert lines[0] == "P3", lines[0]
    w, h, mx = map(int, lines[1].split())
    assert mx == 255
    vals = np.array(" ".join(lines[2:]).split(), dtype=np.int64)
    assert vals.size == w * h * 3 and vals.min() >= 0 and vals.max() <= 255
    return w, h, vals.astype(np.uint8).reshape(h, w, 3)


def main() -> int:
    out = REPO / "tests/golden/ppm"
    out.mkdir(parents=True, exist_ok=True)
    manifest = {}
    for name in GOLDENS:
        raw = (REF / "tests/golden" / f"{name}.ppm").read_bytes()
        w, h, img = parse_p3(raw.decode())
        (out / f"{name}.u8.gz").write_bytes(gzip.compress(img.tobytes(), 9, mtime=0))
        manifest[name] = {"width": w, "height": h, "md5_ppm": hashlib.md5(raw).hexdigest()}
    (out / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=True) + "\n")
    adir = REPO / "hello-raytracing_amd/assets"
    adir.mkdir(parents=True, exist_ok=True)
    for name in ASSETS:
        raw = (REF / "src/assets" / f"{name}.obj").read_bytes()
        (adir / f"{name}.obj.gz").write_bytes(gzip.compress(raw, 9, mtime=0))
    print(f"wrote {len(GOLDENS)} goldens, {len(ASSETS)} assets")
    return 0


if __name__ == "__main__":
    sys.exit(main())
