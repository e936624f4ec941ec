"""Each launch folds the launch before it (rt_params.fold 3, RT_FOLD_NEXT; rt_kernels.hip fold_prev_tiles; DESIGN.md §6
Round 6).

A sample-buffer draw of two or more launches of the suspendable-walk kernels alternates two sample buffers: launch k
writes buffer k % 2 while 1 in 64 of its waves first fold buffer (k - 1) % 2 into the image, tile by tile from a
counter, and k_accumulate folds the last launch only. The folds stay in frame order (launch k's colours are folded
inside launch k + 1, before launch k + 1's own), so images and query counts must equal the draw that runs k_accumulate
after every launch (fold 1) and the oracle's. The cases force many short launches (a 1 MiB budget: 40 frames of 96 x 64
in launches of 14 + 14 + 12) through k_trace_split (culling BVH) and k_trace_split_tris (triangle and mixed programs),
with the tile order learnt in every launch, stealing, and back-to-back draws read in between.
"""
import numpy as np
import pytest

import hrt
import scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if hrt.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on an MI355X box (there is no CPU fallback)")


def _suzanne_tris(w, h, frames):
    scene = hrt.SceneTris.new_suzane(w, h)
    return scenes.SceneDef("suzane", hrt.RT_MODE_TRIS, w, h, scene.camera, bvh=scene.tris_bvh.view(), frames=frames)


CASES = {
    "c3_bvh": lambda: scenes.config_c3(96, 64, 40),
    "c4_mixed": lambda: scenes.config_c4(96, 64, 40),
    "c5_mixed": lambda: scenes.config_c5(96, 64, 40),
    "tris": lambda: _suzanne_tris(96, 64, 40),
}


def _draws(sd, draws=1, **params):
    """`draws` consecutive draws of sd.frames frames (the frame count carries on), the image read after each."""
    r = scenes.make_renderer(sd)
    r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, queue_budget_mb=1, job_frames=4, **params)
    imgs, stats = [], []
    for _ in range(draws):
        r.draw_frames(sd.frames, 1000, 10)
        imgs.append(r.read_image())
        stats.append(r.stats())
    return imgs, stats


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("knobs", ["order_learnt_every_launch", "steal", "plain"])
def test_fold_by_next_launch_equals_fold_after_each(case, knobs):
    sd = CASES[case]()
    extra = {"order_learnt_every_launch": {"cost_order": 3}, "steal": {"steal": 2}, "plain": {"cost_order": 1}}[knobs]
    a, sa = _draws(sd, draws=2, fold=hrt.RT_FOLD_BUFFER, **extra)
    b, sb = _draws(sd, draws=2, fold=hrt.RT_FOLD_NEXT, **extra)
    for k in range(2):
        assert sa[k].fold_ring == 0 and sb[k].fold_ring == 2, (sa[k].fold_ring, sb[k].fold_ring)
        n = sb[k].trace_launches
        assert n == 3 and sa[k].trace_launches == n, n
        assert sa[k].launches == 2 * n and sb[k].launches == n + 1, (sa[k].launches, sb[k].launches)
        assert sb[k].queries == sa[k].queries and sb[k].kernel == sa[k].kernel
        assert (sb[k].node_tests, sb[k].tri_tests) == (sa[k].node_tests, sa[k].tri_tests)
        assert sb[k].fold_bytes == 2 * sa[k].fold_bytes
        np.testing.assert_array_equal(b[k].view(np.uint32), a[k].view(np.uint32), err_msg=f"{case} {knobs} draw {k}")


@pytest.mark.parametrize("case", ["c3_bvh", "c5_mixed"])
def test_fold_by_next_launch_equals_the_oracle(case):
    """A cold renderer (its first launch learns the tile order) against the oracle, rays counted in-kernel."""
    sd = CASES[case]()
    (img,), (st,) = _draws(sd, fold=hrt.RT_FOLD_NEXT)
    assert st.fold_ring == 2 and st.trace_launches == 3
    ref, q = scenes.oracle_render(sd)
    np.testing.assert_array_equal(img.view(np.uint32), ref.view(np.uint32), err_msg=case)
    assert st.queries == q


def test_fold_auto_follows_the_budget_and_the_kernel():
    """fold 0 (auto) folds by the next launch with the automatic colour budget when a suspendable-walk draw takes two
    or more launches (C3 at 1080p x 700 frames: 352 + 348), not under an explicit budget, not in one launch, and not
    for k_trace (the linear scan's register allocation would lose a wave: fold 3 folds after each launch there)."""
    sd = scenes.config_c3(1920, 1080, 700)
    r = scenes.make_renderer(sd)
    r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE)
    r.draw_frames(sd.frames, 1000, 10)
    st = r.stats()
    assert (st.trace_launches, st.launches, st.fold_ring) == (2, 3, 2), (st.trace_launches, st.launches, st.fold_ring)
    want = r.read_image()
    for params, launches in (({"queue_budget_mb": 16384}, 2), ({"fold": hrt.RT_FOLD_BUFFER}, 2),
                             ({"queue_budget_mb": 32768}, 1)):
        r2 = scenes.make_renderer(sd)
        r2.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, **params)
        r2.draw_frames(sd.frames, 1000, 10)
        st2 = r2.stats()
        assert st2.trace_launches == launches and st2.fold_ring == 0, (params, st2.trace_launches, st2.fold_ring)
        np.testing.assert_array_equal(r2.read_image().view(np.uint32), want.view(np.uint32), err_msg=str(params))
    lin = scenes.config_c2(96, 64, 40)
    (img,), (st,) = _draws(lin, fold=hrt.RT_FOLD_NEXT)
    assert st.kernel.decode().startswith("k_trace<") and st.fold_ring == 0 and st.launches == 2 * st.trace_launches
    (img1,), _ = _draws(lin, fold=hrt.RT_FOLD_BUFFER)
    np.testing.assert_array_equal(img.view(np.uint32), img1.view(np.uint32))
    with pytest.raises(hrt.RtError):
        r.set_params(fold=4)
