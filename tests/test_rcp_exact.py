"""The refined reciprocal's exactness claim (rt_device.hpp rcp_rn_mid), by enumeration on the host.

rcp_rn_mid(l) = fma(fma(-l, r0, 1), r0, r0) with r0 = v_rcp_f32(l) replaces the IEEE `1.0f / l` of the triangle
test's 1/det (intersect_triangle, shader_tris.wgsl:161-202) and of the heap walk's 1/d (intersect_node). For every
significand and every r0 within 1 ulp of 1 / l, the step must give the correctly rounded reciprocal; the single
exception is the tie r0 = 1/2 under the all-ones significand. Whether v_rcp_f32 ever returns that r0 is what the
GPU self-check (`rt_check_exact_math`, test_gpu_parity.py) settles, over every significand.
"""
import pathlib
import shutil
import subprocess

import pytest

HERE = pathlib.Path(__file__).resolve().parent


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_one_newton_step_rounds_correctly(tmp_path):
    exe = tmp_path / "rcp_exact_enum"
    subprocess.run(["gcc", "-O2", "-std=c99", "-ffp-contract=off", "-o", str(exe), str(HERE / "rcp_exact_enum.c"),
                    "-lm"], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    cases, bad = map(int, out[0].split())
    assert cases == 2 * (1 << 23) + 1
    # the only failure: l = 2 - 2^-23 (all-ones significand), r0 = 0.5 -> r1 = 0.5 (a tie), RN(1 / l) = 0.5 + 2^-24
    assert bad == 1, out[: 8]
    m, r0, r1, ref = (int(v, 16) for v in out[1].split())
    assert (m, r0, r1, ref) == (0x7FFFFF, 0x3F000000, 0x3F000000, 0x3F000001)
