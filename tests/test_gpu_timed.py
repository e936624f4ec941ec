"""The timed configurations pinned end to end against the oracle.

bench.py times compositions the other parity tests cover only in parts: C3 at 1024 frames drawn in three balanced
sample-buffer launches (352 + 352 + 320 frames) by the uncounted k_trace_split, with the EMA switch at frame 1000
(shader_sphere.wgsl:264-271: the weight stops at 1 / (SAMPLE_FRAME + 1)) inside the third launch's k_accumulate fold;
C4 at 512 frames in one launch; C5 at 4096 frames in twelve launches of 342 frames. Each test draws exactly that —
the renderer set up by bench.py's own `timed_knobs` and frame protocol — and compares whole rows bit for bit with the
oracle at every frame count, and asserts the launch composition the bench line reports (kernel, launches, frames per
launch). Oracle cost on the GPU box's 16 threads: a few seconds per config (oracle work items are 64-column chunks).
"""
import numpy as np
import pytest

import bench
import hrt
import scenes
from hrt.parallel import rank_params

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if hrt.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on an MI355X box (there is no CPU fallback)")


def assert_bits(gpu: np.ndarray, ref: np.ndarray, what: str):
    assert gpu.shape == ref.shape, (what, gpu.shape, ref.shape)
    d = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
    same = gpu.view(np.uint32) == ref.view(np.uint32)
    assert same.all(), f"{what}: {np.size(same) - same.sum()} channels differ (max |d| {np.nanmax(d)})"


def timed_draw(sd, **params):
    """One bench step (bench.py main/step): the one-rank row partition, the timed knobs, reset, draw every frame."""
    r = scenes.make_renderer(sd)
    r.set_params(**rank_params(0, 1, 8), **bench.timed_knobs(**params))
    r.reset_frame_count()
    r.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
    return r, r.read_image(), r.stats()


def test_c3_as_timed_crosses_the_ema_switch_inside_a_launch():
    sd = scenes.config_c3()
    assert (sd.width, sd.height, sd.frames) == (1920, 1080, 1024)
    r, img, st = timed_draw(sd)
    # the composition of the bench line (BENCH_r04: kernel, launch_frames 352, 3 launches per step)
    assert st.kernel.decode() == "k_trace_split<true, false, false>", st.kernel
    assert (st.trace_launches, st.launch_frames, st.fold_ring) == (3, 352, 0), (st.trace_launches, st.launch_frames)
    assert st.box_tests == 0 and st.sphere_tests == 0  # uncounted, as timed
    assert 704 < 1000 < 1024  # frame 1000 is folded by the third launch's k_accumulate
    rows = (7, 536, 3)  # rows 7, 543, 1079
    ref, _ = scenes.oracle_render(sd, rows=rows)
    assert_bits(img[7::536], ref, "C3 timed composition, rows 7 / 543 / 1079 x 1024 frames")
    # the same rows alone, in the same three launches (a 62 MiB budget holds 352 frames of one tile row), give the
    # oracle's ray count too (stealing off: the bench's kernel)
    r2 = scenes.make_renderer(sd)
    r2.set_params(row0=7, row_step=536, row_block=1, **bench.timed_knobs(queue_budget_mb=62, steal=1))
    r2.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
    st2 = r2.stats()
    assert st2.kernel.decode() == "k_trace_split<true, false, false>" and st2.trace_launches == 3
    assert st2.launch_frames == 352
    _, q = scenes.oracle_render(sd, rows=rows)
    assert st2.queries == q
    assert_bits(r2.read_image(), ref, "C3 rows alone, three launches")


def test_c4_as_timed():
    sd = scenes.config_c4()
    assert (sd.width, sd.height, sd.frames) == (1920, 1080, 512)
    r, img, st = timed_draw(sd)
    assert st.kernel.decode() == "k_trace_split_tris<2, 1, 3, false>", st.kernel
    assert (st.trace_launches, st.launch_frames, st.fold_ring) == (1, 512, 0)
    ref, _ = scenes.oracle_render(sd, rows=(452, 160, 2))  # rows 452, 612: Suzanne and the ground
    assert_bits(img[452:613:160], ref, "C4 timed composition, rows 452 / 612 x 512 frames")


def test_c5_as_timed_in_twelve_launches():
    """C5's full 4K image takes 9 s per step; its timed composition — twelve sample-buffer launches of 342 frames (the
    auto budget's 32 GiB cap), frame 1000 inside the third, the kernel k_trace_split_tris<2, 4, 3, false> — is drawn on
    one row with a 121 MiB budget (the same 342-frame launches) and stealing off (a one-row draw has few jobs per wave,
    which would turn the auto stealing on). A 512-column window of the row against the oracle at all 4096 frames."""
    sd = scenes.config_c5()
    assert (sd.width, sd.height, sd.frames) == (3840, 2160, 4096)
    r = scenes.make_renderer(sd)
    r.set_params(row0=1080, row_step=2160, row_block=1, **bench.timed_knobs(queue_budget_mb=121, steal=1))
    r.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
    img, st = r.read_image(), r.stats()
    assert st.kernel.decode() == "k_trace_split_tris<2, 4, 3, false>", st.kernel
    assert (st.trace_launches, st.launch_frames, st.fold_ring) == (12, 342, 0), (st.trace_launches, st.launch_frames)
    x0, nx = 1664, 512
    ref, _ = scenes.oracle_render(sd, rows=(1080, 1, 1), x0=x0, nx=nx)
    assert_bits(img[:, x0:x0 + nx], ref, "C5 timed composition, row 1080, columns 1664-2175 x 4096 frames")
