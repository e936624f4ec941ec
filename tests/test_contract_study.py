"""The float-contract study of the golden residuals (tests/golden/contract_study.py).

The reference's golden images come from an unknown GPU whose shader compiler may fuse or reassociate float
operations differently from this build's contract (oracle/rt_oracle.c, contract 0). The study renders the
seven golden scenes under ten contracts (ORACLE_CONTRACT 0-5: the build's; no FMA; every a*b+c fused;
normalize as v * (1 / |v|); 2 + 3; every division as a * (1 / b); 6-9, VERDICT r3: the hardware-approximate forms
a shader compiler may emit — pow(x, 5) as exp2(5 log2 x), normalize through a 1-ulp rsq, tan as sin / cos, all
three) and stores the table in tests/golden/contract_study.json. These tests pin its findings and re-render a band
of one golden under every contract:

* no alternative contract matches the non-glass goldens materially better than the build's (the residual is
  not a contract choice this build could make);
* the residual is at float-contract noise level: about half of the build's mismatched channels change under
  some other contract, and every contract leaves the same order of mismatches (1e-4 of the channels);
* the hardware-approximate forms do not close it either: pow through exp2 / log2 and tan through sin / cos change
  no non-glass golden by more than 1e-5 of its channels; the 1-ulp rsq normalize lowers the largest non-glass
  difference of lambertian_materials and metal_materials from 5 to 3 but matches fewer channels exactly
  (99.991 vs 99.994 %, 99.987 vs 99.992 %) and the glass scenes worse (mean |du8| 0.482 vs 0.422 %), so the
  oracle and the kernels keep contract 0.
"""
import json
from pathlib import Path

import numpy as np

import scenes

STUDY = json.loads((Path(__file__).resolve().parent / "golden" / "contract_study.json").read_text())
NON_GLASS = ["lambertian_materials", "metal_materials", "camera_position", "depth_of_field", "shadow_rendering"]


def test_study_table_no_contract_closes_the_residual():
    assert set(STUDY["contracts"]) == {str(c) for c in range(10)}
    for name in NON_GLASS:
        per = STUDY["scenes"][name]
        c0 = per["0"]["exact_u8"]
        assert c0 >= 0.9998, (name, c0)
        best = max(per[c]["exact_u8"] for c in per)
        assert best - c0 <= 2e-5, (name, {c: per[c]["exact_u8"] for c in per})  # <= 16 of 786432 channels
        assert all(per[c]["max_abs_du8"] <= 5 for c in per), name
        # the build's mismatches are mostly off-edge, none reach glass, and many are contract-fragile
        assert per["0"]["glass"] == 0
        assert per["0"]["mismatched_channels_fragile"] * 3 >= per["0"]["mismatched_channels"], name


def test_hardware_approximate_forms_do_not_close_the_residual():
    """Contracts 6-9 against the build's: no exact-match gain on a non-glass golden, the rsq
    normalize's smaller maximum bought with more mismatched channels, and no glass mean below the build's but
    contract 5's 0.004 % (the reciprocal division, not a hardware-approximate form)."""
    for name in NON_GLASS:
        per = STUDY["scenes"][name]
        c0 = per["0"]["exact_u8"]
        for c in ("6", "8"):
            assert abs(per[c]["exact_u8"] - c0) <= 1e-5, (name, c)
        assert max(per[c]["exact_u8"] for c in ("6", "7", "8", "9")) <= c0 + 1e-5, name
    for name in ("lambertian_materials", "metal_materials"):
        per = STUDY["scenes"][name]
        assert per["7"]["max_abs_du8"] == 3 < per["0"]["max_abs_du8"] == 5, name
        assert per["7"]["exact_u8"] < per["0"]["exact_u8"], name
    for name in ("dielectric_materials", "complex_scene"):
        per = STUDY["scenes"][name]
        m0 = per["0"]["mean_abs_du8_pct"]
        assert min(per[c]["mean_abs_du8_pct"] for c in ("6", "7", "8", "9")) >= m0 - 1e-6, name
        assert per["7"]["mean_abs_du8_pct"] > m0, name


def test_contracts_render_a_golden_band():
    """Rows 200-223 of camera_position (512 x 512, 100 frames) under the ten contracts: each matches the golden
    on >= 99.9 % of the band's channels, they are distinct builds (contract 1's floats differ from contract
    0's), and contract 0 is the committed build's oracle."""
    sd = scenes.golden_scene("camera_position")
    golden = scenes.load_golden_u8("camera_position")[200:224]
    imgs = {}
    for c in range(10):
        img, _ = scenes.oracle_render(sd, frames=scenes.GOLDEN_FRAMES, rows=(200, 1, 24), contract=c)
        imgs[c] = img
        u8 = scenes.to_u8(img)
        d = np.abs(u8.astype(np.int32) - golden.astype(np.int32))
        assert np.mean(d == 0) >= 0.999 and d.max() <= 3, (c, np.mean(d == 0), d.max())
    assert not np.array_equal(imgs[0].view(np.uint32), imgs[1].view(np.uint32))
    ref, _ = scenes.oracle_render(sd, frames=scenes.GOLDEN_FRAMES, rows=(200, 1, 24))
    np.testing.assert_array_equal(imgs[0].view(np.uint32), ref.view(np.uint32))
