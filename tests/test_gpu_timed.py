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
from hrt.parallel import owned_rows, rank_params

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


def timed_draw(sd, rank=0, world=1, block=8, warmup=1, **params):
    """One bench step as bench.run_leg times it: this rank's row share, the timed knobs, `warmup` counting steps (they
    learn the tiles' cost order, rt_params.cost_order), then reset and draw every frame uncounted."""
    r = scenes.make_renderer(sd)
    r.set_params(**rank_params(rank, world, block), **bench.timed_knobs(**params))
    for _ in range(warmup):  # (bench.run_leg counting_step)
        r.set_params(count_tests=1)
        r.reset_frame_count()
        r.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
        r.set_params(count_tests=0)
    r.reset_frame_count()
    r.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
    return r, r.read_image(), r.stats()


def composition(st) -> tuple:
    """What the bench line reports of a timed step's launches."""
    return st.kernel.decode(), st.trace_launches, st.launch_frames, st.ordered_launches, st.fold_ring


def local_row(rank, world, block, height, row) -> int:
    rows = list(owned_rows(block * rank, world, height, block))
    return rows.index(row)


def test_c3_as_timed_crosses_the_ema_switch_inside_a_launch():
    sd = scenes.config_c3()
    assert (sd.width, sd.height, sd.frames) == (1920, 1080, 1024)
    r, img, st = timed_draw(sd)
    # the composition of the bench line (kernel, 3 launches of 352 frames per step, all three dealt in the cost order
    # the warmup step learnt, two sample buffers: launches 2 and 3 fold the launch before, k_accumulate the third)
    assert composition(st) == ("k_trace_split<true, false, false, false>", 3, 352, 3, 2), composition(st)
    assert st.launches == 4, st.launches
    assert st.box_tests == 0 and st.sphere_tests == 0  # uncounted, as timed
    assert 704 < 1000 < 1024  # frame 1000 is folded by the third launch's k_accumulate
    rows = (7, 536, 3)  # rows 7, 543, 1079
    ref, _ = scenes.oracle_render(sd, rows=rows)
    assert_bits(img[7::536], ref, "C3 timed composition, rows 7 / 543 / 1079 x 1024 frames")
    # the same rows alone, in the same three launches (a 62 MiB budget holds 352 frames of one tile row), give the
    # oracle's ray count too (stealing off: the bench's kernel; each launch folded by the next, as timed)
    r2 = scenes.make_renderer(sd)
    r2.set_params(row0=7, row_step=536, row_block=1,
                  **bench.timed_knobs(queue_budget_mb=62, steal=1, fold=hrt.RT_FOLD_NEXT))
    r2.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
    st2 = r2.stats()
    assert st2.kernel.decode() == "k_trace_split<true, false, false, false>" and st2.trace_launches == 3
    assert st2.fold_ring == 2
    assert st2.launch_frames == 352
    _, q = scenes.oracle_render(sd, rows=rows)
    assert st2.queries == q
    assert_bits(r2.read_image(), ref, "C3 rows alone, three launches")


def test_c4_as_timed():
    sd = scenes.config_c4()
    assert (sd.width, sd.height, sd.frames) == (1920, 1080, 512)
    r, img, st = timed_draw(sd, block=4)
    assert composition(st) == ("k_trace_split_tris<2, 1, 3, false>", 1, 512, 1, 0), composition(st)
    ref, _ = scenes.oracle_render(sd, rows=(452, 160, 2))  # rows 452, 612: Suzanne and the ground
    assert_bits(img[452:613:160], ref, "C4 timed composition, rows 452 / 612 x 512 frames")


def test_c5_as_timed_in_twelve_launches():
    """C5's full 4K image takes 9 s per step; its timed composition — twelve sample-buffer launches of 342 frames (the
    auto budget's 32 GiB cap), frame 1000 inside the third, the kernel k_trace_split_tris<2, 4, 3, false> — is drawn on
    one row with a 121 MiB budget (the same 342-frame launches) and stealing off (a one-row draw has few jobs per wave,
    which would turn the auto stealing on), each launch folded by the next as the auto budget's are. A 512-column
    window of the row against the oracle at all 4096 frames."""
    sd = scenes.config_c5()
    assert (sd.width, sd.height, sd.frames) == (3840, 2160, 4096)
    r = scenes.make_renderer(sd)
    r.set_params(row0=1080, row_step=2160, row_block=1,
                 **bench.timed_knobs(queue_budget_mb=121, steal=1, fold=hrt.RT_FOLD_NEXT))
    r.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
    img, st = r.read_image(), r.stats()
    assert st.kernel.decode() == "k_trace_split_tris<2, 4, 3, false>", st.kernel
    assert (st.trace_launches, st.launch_frames, st.fold_ring) == (12, 342, 2), composition(st)
    x0, nx = 1664, 512
    ref, _ = scenes.oracle_render(sd, rows=(1080, 1, 1), x0=x0, nx=nx)
    assert_bits(img[:, x0:x0 + nx], ref, "C5 timed composition, row 1080, columns 1664-2175 x 4096 frames")


def test_c3_rank_share_as_timed_at_eight_ranks():
    """The share the driver's 8-GPU run times on rank 4: rows dealt in 8-row blocks, one 1024-frame
    launch, dealt in the cost order the counting warmup step learnt (no stealing once learnt). Global row 547
    (local row 67) against the oracle at all 1024 frames."""
    sd = scenes.config_c3()
    r, img, st = timed_draw(sd, rank=4, world=8, block=8)
    assert composition(st) == ("k_trace_split<true, false, false, false>", 1, 1024, 1, 0), composition(st)
    k = local_row(4, 8, 8, sd.height, 547)
    ref, _ = scenes.oracle_render(sd, rows=(547, 1, 1))
    assert_bits(img[k:k + 1], ref, "C3 rank 4 of 8, row 547 x 1024 frames")


def test_c4_rank_share_as_timed_at_eight_ranks():
    """C4's 8-rank share (4-row blocks, bench.ROW_BLOCK): rank 3, global row 524 (Suzanne) at all 512 frames."""
    sd = scenes.config_c4()
    r, img, st = timed_draw(sd, rank=3, world=8, block=4)
    assert composition(st) == ("k_trace_split_tris<2, 1, 3, false>", 1, 512, 1, 0), composition(st)
    k = local_row(3, 8, 4, sd.height, 524)
    ref, _ = scenes.oracle_render(sd, rows=(524, 1, 1))
    assert_bits(img[k:k + 1], ref, "C4 rank 3 of 8, row 524 x 512 frames")


def test_c2_as_timed():
    """C2 (the linear sphere scan, k_trace) at 256 spp: one launch, raster order (cost order is for the suspendable-walk
    kernels' full images and the ranks' shares). Rows 200 (the three spheres) and 500 (the ground) at all frames."""
    sd = scenes.config_c2()
    assert (sd.width, sd.height, sd.frames) == (1280, 720, 256)
    r, img, st = timed_draw(sd)
    assert composition(st) == ("k_trace<0, 1, false>", 1, 256, 0, 0), composition(st)
    ref, _ = scenes.oracle_render(sd, rows=(200, 300, 2))
    assert_bits(img[200:501:300], ref, "C2 timed composition, rows 200 / 500 x 256 frames")
