"""Float-contract study of the residual mismatches against the reference's golden images.

The reference's goldens (tests/golden/*.ppm) come from an unknown GPU through naga, whose compiler may fuse or
reassociate float operations. The build's contract (oracle/rt_oracle.c, contract 0) matches the non-glass
goldens on 99.99 % of u8 channels; this study renders the seven golden scenes (512 x 512, 100 frames,
time 1000 + 10 i) with the oracle under ten contracts (0-5: fusion / division / normalize forms; 6-9: the
hardware-approximate forms a GPU shader compiler may emit for pow, normalize and tan) and, for contract 0, sorts
every channel that differs
from the golden by where it lies:

* edge: the pixel sits on a silhouette, shadow boundary or texture edge — some 4-neighbour differs from it by
  more than 16/255 in the golden image (a sample whose jittered primary ray lands on the other side of an edge
  changes the pixel by a whole colour step / 100);
* glass: the pixel's primary rays reach a dielectric sphere in the oracle render (chaotic);
* interior: neither.
It also reports how many of those channels are float-fragile: their u8 value changes under at least one of
the other contracts — the mismatch then depends on the reference GPU's unknown contract.

usage: python tests/golden/contract_study.py [--out tests/golden/contract_study.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
for p in (ROOT, ROOT / "hello-raytracing_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))

import scenes  # noqa: E402

CONTRACTS = {0: "build contract (FMA in dot / disc / point_on_ray; v / sqrt)", 1: "no FMA at all",
             2: "contract 0 + every a*b+c fused", 3: "contract 0 + normalize as v * (1 / sqrt)",
             4: "contracts 2 + 3", 5: "every division by a computed value as a * (1 / b)",
             6: "contract 0 + pow(x, 5) as exp2(5 log2 x)", 7: "contract 0 + normalize as v * rsq(v.v), 1-ulp rsq",
             8: "contract 0 + tan(fov/2) as sin * (1 / cos) in f32", 9: "contracts 6 + 7 + 8"}


def edge_mask(golden: np.ndarray) -> np.ndarray:
    g = golden.astype(np.int32)
    m = np.zeros(g.shape[:2], dtype=bool)
    for axis, shift in ((0, 1), (0, -1), (1, 1), (1, -1)):
        d = np.abs(g - np.roll(g, shift, axis=axis)).max(axis=2)
        m |= d > 16
    return m


def glass_mask(name: str) -> np.ndarray:
    """Pixels whose one-bounce render differs when the dielectric spheres are made lambertian (the primary
    ray of some sample reaches glass)."""
    sd = scenes.golden_scene(name)
    sd.frames, sd.bounces = 4, 2
    a, _ = scenes.oracle_render(sd)
    sp = sd.spheres.copy()
    glass = sp["material"]["kind"] == 3
    if not glass.any():
        return np.zeros((sd.height, sd.width), dtype=bool)
    sp["material"]["kind"][glass] = 1
    sd.spheres = sp
    b, _ = scenes.oracle_render(sd)
    return (a != b).any(axis=2)


def study(names=None):
    names = names or list(scenes.GOLDEN_NAMES)
    out = {}
    for name in names:
        golden = scenes.load_golden_u8(name)
        sd = scenes.golden_scene(name)
        per = {}
        u8 = {}
        for c in CONTRACTS:
            img, _ = scenes.oracle_render(sd, frames=scenes.GOLDEN_FRAMES, contract=c)
            u8[c] = scenes.to_u8(img)
            d = np.abs(u8[c].astype(np.int32) - golden.astype(np.int32))
            per[c] = {"exact_u8": float(np.mean(d == 0)), "mismatched_channels": int((d != 0).sum()),
                      "max_abs_du8": int(d.max()), "mean_abs_du8_pct": float(d.mean() / 255 * 100)}
            if c == 0:
                bad = (d != 0).any(axis=2)
                e, gl = edge_mask(golden), glass_mask(name)
                per[c]["mismatched_pixels"] = int(bad.sum())
                per[c]["edge"] = int((bad & e & ~gl).sum())
                per[c]["glass"] = int((bad & gl).sum())
                per[c]["interior"] = int((bad & ~e & ~gl).sum())
                per[c]["edge_pixels_in_image"] = float(e.mean())
        fragile = np.zeros_like(golden, dtype=bool)
        for c in CONTRACTS:
            fragile |= u8[c] != u8[0]
        bad0 = u8[0] != golden
        per[0]["mismatched_channels_fragile"] = int((bad0 & fragile).sum())
        per[0]["fragile_channels_in_image"] = int(fragile.sum())
        i = np.unravel_index(np.argmax(np.abs(u8[0].astype(np.int32) - golden.astype(np.int32))), golden.shape)
        per[0]["worst_channel"] = {"y": int(i[0]), "x": int(i[1]), "c": int(i[2]), "golden": int(golden[i]),
                                   "oracle": int(u8[0][i]), "fragile": bool(fragile[i])}
        out[name] = per
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "tests" / "golden" / "contract_study.json"))
    a = ap.parse_args()
    res = study()
    Path(a.out).write_text(json.dumps({"contracts": CONTRACTS, "scenes": res}, indent=1))
    print("| golden | " + " | ".join(f"c{c} exact / max / mean" for c in CONTRACTS)
          + " | c0 mismatched px: edge / glass / interior | c0 mismatched channels float-fragile |")
    print("|---|" + "---|" * (len(CONTRACTS) + 2))
    for name, per in res.items():
        cells = [f"{per[c]['exact_u8'] * 100:.3f} % / {per[c]['max_abs_du8']} / {per[c]['mean_abs_du8_pct']:.3f} %"
                 for c in CONTRACTS]
        p0 = per[0]
        print(f"| {name} | " + " | ".join(cells) + f" | {p0['edge']} / {p0['glass']} / {p0['interior']} | "
              f"{p0['mismatched_channels_fragile']} of {p0['mismatched_channels']} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
