"""The CPU oracle against the reference's own golden images (pins the oracle; no GPU needed).

Goldens: tests/golden/ppm/*.u8.gz, converted from the reference's tests/golden/*.ppm by
tests/golden/make_fixtures.py; scene definitions restate tests/rendering_tests.rs:134-509. The goldens were
rendered with 100 frames at time 1000 + 10 i, on an unknown GPU whose float behaviour
(FMA contraction, sqrt/pow/tan precision) cannot be reproduced, so the bar is statistical:
  * the reference harness's own metric: mean |du8| <= 2 % of 255 (rendering_tests.rs:11, :84-131) — all 7;
  * non-glass scenes: >= 99.98 % of u8 channels bit-exact, max |du8| <= 5 — the float-noise floor the
    contract study shows irreducible by any of six float contracts (test_contract_study.py);
  * glass scenes (dielectric_materials, complex_scene): mean |du8| <= 0.6 % (refraction re-hit chaos:
    intersect_sphere keeps only the near root and refracted rays start on the surface).
"""
import numpy as np
import pytest

import hrt
import scenes


@pytest.mark.parametrize("name", scenes.GOLDEN_NAMES)
def test_oracle_matches_reference_golden(name):
    sd = scenes.golden_scene(name)
    img, q = scenes.oracle_render(sd)
    u8 = scenes.to_u8(img)
    golden = scenes.load_golden_u8(name)
    d = np.abs(u8.astype(np.int32) - golden.astype(np.int32))
    mean_pct = d.mean() / 255.0 * 100.0
    exact = np.mean(d == 0)
    # the reference harness, through the product's own render_ppm + compare_ppm_images
    pct = hrt.compare_ppm_images(hrt.ppm_from_image(img, 512, 512), scenes.ppm_text_from_u8(golden), 2.0)
    assert abs(pct - mean_pct) < 1e-3
    assert q > 512 * 512 * 100  # at least one query per sample
    if name in scenes.GLASS_GOLDENS:
        assert mean_pct <= 0.6, (name, mean_pct, exact)
    else:
        assert exact >= 0.9998 and d.max() <= 5, (name, exact, d.max())


def test_orphan_golden_materials_is_unpinned():
    """materials.ppm has no generator in the reference's tests: we only check it loads (unpinned)."""
    g = scenes.load_golden_u8("materials")
    assert g.shape == (512, 512, 3)


def test_one_frame_would_fail_the_reference_threshold():
    """Documents SURVEY §0 F4: at TEST_FRAMES = 1 (as checked in) dielectric fails the 2 % bar, so the
    goldens must have been made with 100 frames. Uses a 128-row band to stay fast."""
    sd = scenes.golden_scene("dielectric_materials")
    img, _ = scenes.oracle_render(sd, frames=1, rows=(192, 1, 128))
    golden = scenes.load_golden_u8("dielectric_materials")[192:320]
    d = np.abs(scenes.to_u8(img).astype(np.int32) - golden.astype(np.int32))
    assert d.mean() / 255.0 * 100.0 > 2.0
