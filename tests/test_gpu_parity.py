"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle and the reference's goldens.

Tolerance (BASELINE.json north star): per-channel float max |d| <= 1e-3 between the HIP image and the
oracle image on the same scene, seeds and frames. The build's float contract makes the two bit-identical
by construction; the tests also report the bit-exact fraction and require it to be 1.0
on every scene, since one differing ulp on a glass scene diverges the path and breaks the 1e-3 bound anyway.
Integer outputs (closest-hit query counts) must match exactly.
"""
import numpy as np
import pytest
import torch

import hrt
import scenes

pytestmark = pytest.mark.gpu

TOL = 1e-3


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if hrt.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on an MI355X box (there is no CPU fallback)")


def assert_parity(gpu: np.ndarray, ref: np.ndarray, what: str):
    assert gpu.shape == ref.shape, what
    d = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
    bad = ~(d <= TOL)
    exact = np.mean(gpu.view(np.uint32) == ref.view(np.uint32))
    assert not bad.any(), f"{what}: {bad.sum()} channels beyond {TOL} (max {np.nanmax(d)}), bit-exact {exact:.6f}"
    assert exact == 1.0, f"{what}: within tolerance but only {exact:.6f} bit-exact"


def render_reference_protocol(sd: scenes.SceneDef, frames: int):
    """tests/rendering_tests.rs:14-28 flow: init, then frames x {set_time(1000 + 10 i); draw()}."""
    scene = hrt.SceneSphere(hrt.Renderer(sd.width, sd.height, hrt.RT_MODE_SPHERE), sd.camera,
                            [s for s in sd.spheres])
    scene.init()
    for i in range(frames):
        scene.set_time(1000 + i * 10)
        scene.draw()
    return scene


@pytest.mark.parametrize("name", scenes.GOLDEN_NAMES)
def test_golden_scene_hip_vs_oracle_and_golden(name):
    sd = scenes.golden_scene(name)
    scene = render_reference_protocol(sd, scenes.GOLDEN_FRAMES)
    img = scene.renderer.read_image()
    stats = scene.renderer.stats()
    # oracle on every 4th row (pixels are independent; global coordinates)
    ref, q = scenes.oracle_render(sd, rows=(0, 4, 128))
    assert_parity(img[0::4], ref, name)
    # reference harness: render_ppm + compare_ppm_images(2 %) against the reference golden
    golden = scenes.load_golden_u8(name)
    golden_ppm = scenes.ppm_text_from_u8(golden)
    pct = hrt.compare_ppm_images(hrt.render_ppm(scene.renderer), golden_ppm, 2.0)
    u8 = scenes.to_u8(img)
    exact = np.mean(u8 == golden)
    if name in scenes.GLASS_GOLDENS:
        assert pct <= 0.6, (name, pct)
    else:
        assert exact >= 0.999 and pct <= 0.01, (name, exact, pct)
    assert stats.samples == 512 * 512  # last draw() = one frame


@pytest.mark.parametrize("name", scenes.GOLDEN_NAMES)
def test_golden_scene_full_draw_sample_queue(name):
    """The same golden scenes at full size drawn as one 100-frame draw: the sample queue with the
    suspendable-walk kernel (100 slots -> culling BVH) equals the per-frame reference protocol bit for bit."""
    sd = scenes.golden_scene(name)
    per_frame = render_reference_protocol(sd, scenes.GOLDEN_FRAMES).renderer.read_image()
    r = scenes.make_renderer(sd)
    r.draw_frames(scenes.GOLDEN_FRAMES, 1000, 10)
    st = r.stats()
    assert st.schedule == hrt.RT_SCHEDULE_QUEUE and st.suspend_below > 0 and st.variant == 4
    np.testing.assert_array_equal(r.read_image().view(np.uint32), per_frame.view(np.uint32))
    # the fold ring (a 16 MiB budget: 512 slots of 32 frames for 4096 tiles x 4 jobs) gives the same bits
    r = scenes.make_renderer(sd)
    r.set_params(queue_budget_mb=16)
    r.draw_frames(scenes.GOLDEN_FRAMES, 1000, 10)
    assert r.stats().fold_ring == 1
    np.testing.assert_array_equal(r.read_image().view(np.uint32), per_frame.view(np.uint32))


@pytest.mark.parametrize("schedule", [1, 2])
def test_orbit_camera_uniform_vs_oracle(schedule):
    """The interactive app's camera path: OrbitCamera::to_uniform (camera_controller.rs:116-129, w = 0 basis,
    focal 10, blur 0) uploaded through rt_set_camera as Renderer::update_camera_uniform does
    (renderer.rs:330-334): the 4-component make_ray normalise acts in 3-D and the image matches the oracle."""
    sd = scenes.golden_scene("complex_scene", 96, 64)
    cam = hrt.OrbitCamera(sd.width / sd.height, radius=7.0, theta=0.9, phi=1.2)
    cam.target = np.array([0.0, 0.0, -5.0], dtype=np.float32)
    cam.update_position()
    sd.camera = cam.to_uniform()
    assert float(sd.camera["direction"][3]) == 0.0 and float(sd.camera["params"][0]) == 10.0
    sd.frames = 6
    r = scenes.make_renderer(sd)
    r.set_params(schedule=schedule)
    r.draw_frames(sd.frames, 1000, 10)
    img = r.read_image()
    ref, q = scenes.oracle_render(sd)
    assert_parity(img, ref, f"orbit camera, schedule {schedule}")
    assert r.stats().queries == q


def test_draw_frames_equals_per_frame_draws():
    sd = scenes.golden_scene("complex_scene", 96, 64)
    a = render_reference_protocol(sd, 12).renderer.read_image()
    for schedule in (hrt.RT_SCHEDULE_TILES, hrt.RT_SCHEDULE_QUEUE):
        r = scenes.make_renderer(sd)
        r.set_params(frames_per_launch=5, schedule=schedule)  # tiles: 3 launches, 5 + 5 + 2
        r.draw_frames(12, 1000, 10)
        assert r.frame_count == 12 and r.stats().schedule == schedule
        np.testing.assert_array_equal(r.read_image().view(np.uint32), a.view(np.uint32))


def _schedule_cases():
    c3 = scenes.config_c3(90, 53, 5)  # W, H not multiples of the 8x8 tile
    c4 = scenes.config_c4(72, 41, 3)
    golden = scenes.golden_scene("dielectric_materials", 64, 40)
    golden.frames = 6
    return [c3, c4, golden]


@pytest.mark.parametrize("case", [0, 1, 2])
def test_sample_queue_equals_tiles(case):
    """The sample-queue schedule (persistent k_trace + in-order k_accumulate) gives the tiles schedule's
    bits and exact work counters, for sphere, mixed and partitioned renders."""
    sd = _schedule_cases()[case]
    for row0, step in [(0, 1), (1, 3)]:
        out = []
        # (packet 1: the queue's primary rays walk on their own, so the box / sphere test counts are the tiles'; the
        # packet walk's, packet 2, count its union's tests: same bits and queries)
        for schedule, packet in ((hrt.RT_SCHEDULE_TILES, 0), (hrt.RT_SCHEDULE_QUEUE, 1), (hrt.RT_SCHEDULE_QUEUE, 2)):
            r = scenes.make_renderer(sd)
            r.set_params(schedule=schedule, row0=row0, row_step=step, job_frames=3, packet=packet)  # ragged last job
            r.set_frame_count(3)
            r.draw_frames(sd.frames, 2000, 7)
            out.append((r.read_image(), r.stats()))
        (a, sa), (b, sb), (c, sc) = out
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
        np.testing.assert_array_equal(a.view(np.uint32), c.view(np.uint32))
        assert (sa.queries, sa.box_tests, sa.sphere_tests, sa.node_tests, sa.tri_tests) == \
               (sb.queries, sb.box_tests, sb.sphere_tests, sb.node_tests, sb.tri_tests)
        assert (sc.queries, sc.node_tests, sc.tri_tests) == (sa.queries, sa.node_tests, sa.tri_tests)
        assert sb.schedule == hrt.RT_SCHEDULE_QUEUE and sb.samples == sa.samples


def test_auto_schedule_by_draw_size():
    """schedule 0 picks tiles below 1.5 Mi samples per draw and the sample queue from there on."""
    sd = scenes.golden_scene("shadow_rendering", 256, 256)
    r = scenes.make_renderer(sd)
    r.draw_frames(24, 1000, 10)  # 1.5 Mi samples
    assert r.stats().schedule == hrt.RT_SCHEDULE_QUEUE
    r.draw_frames(1, 2000, 10)
    assert r.stats().schedule == hrt.RT_SCHEDULE_TILES
    t = scenes.make_renderer(sd)
    t.set_params(schedule=hrt.RT_SCHEDULE_TILES)
    t.draw_frames(24, 1000, 10)
    t.draw_frames(1, 2000, 10)
    np.testing.assert_array_equal(r.read_image().view(np.uint32), t.read_image().view(np.uint32))


def test_sample_queue_chunks_and_tris_mode():
    """Budgets too small for the sample buffer: fold rings smaller than the draw's jobs (1 and 2 MiB at 320x240:
    32 and 64 job slots of 32 frames for 1200 jobs, so most jobs wait for their slot); a budget holding 320+
    frames: the sample buffer in launches of that many frames; and the triangle program under the queue
    schedule."""
    sd = scenes.golden_scene("metal_materials", 320, 240)
    ref = scenes.make_renderer(sd)
    ref.set_params(schedule=hrt.RT_SCHEDULE_TILES)
    ref.draw_frames(5, 1000, 10)
    for mb in (1, 2):
        r = scenes.make_renderer(sd)
        r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, queue_budget_mb=mb)
        r.draw_frames(5, 1000, 10)
        st = r.stats()
        ring = st.fold_bytes - 4 * 1200 * 3  # minus the per-tile fold words and job -> slot map
        assert st.fold_ring == 1 and st.launches == 1, (st.fold_ring, st.launches)
        assert (mb << 19) < ring <= (mb << 20) + 4 * (4 * 64 * mb + 4), st.fold_bytes
        np.testing.assert_array_equal(r.read_image().view(np.uint32), ref.read_image().view(np.uint32))
    # 320x240 = 1200 tiles, 0.92 MB of colours per frame: 320 MiB hold 364 frames (>= 320: the sample buffer)
    # -> 700 frames in two balanced launches of whole jobs, 352 + 348; the default budget (auto: every frame that
    # 8 GiB holds) and 1000 MiB hold all 700 frames: one launch
    per_frame = 1200 * 64 * 12
    ref = scenes.make_renderer(sd)
    ref.set_params(schedule=hrt.RT_SCHEDULE_TILES)
    ref.draw_frames(700, 1000, 10)
    for mb, nl, chunk in ((320, 2, 352), (None, 1, 700), (1000, 1, 700)):
        r = scenes.make_renderer(sd)
        r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, **({"queue_budget_mb": mb} if mb else {}))
        r.draw_frames(700, 1000, 10)
        st = r.stats()
        assert st.fold_ring == 0 and st.launches == 2 * nl and st.trace_launches == nl, (mb, st.launches)
        assert st.launch_frames == chunk and st.fold_bytes == chunk * per_frame, (mb, st.launch_frames, st.fold_bytes)
        np.testing.assert_array_equal(r.read_image().view(np.uint32), ref.read_image().view(np.uint32))
    scene = hrt.SceneTris.new_suzane(96, 72)
    scene.init()
    sd = scenes.SceneDef("suzane", hrt.RT_MODE_TRIS, 96, 72, scene.camera, bvh=scene.tris_bvh.view(), frames=4)
    imgs = []
    for schedule in (hrt.RT_SCHEDULE_TILES, hrt.RT_SCHEDULE_QUEUE):
        r = scenes.make_renderer(sd)
        r.set_params(schedule=schedule)
        r.draw_frames(4, 1000, 10)
        imgs.append(r.read_image())
    np.testing.assert_array_equal(imgs[0].view(np.uint32), imgs[1].view(np.uint32))
    ref_img, _ = scenes.oracle_render(sd)
    assert_parity(imgs[1], ref_img, "suzane tris, queue schedule")


def _queue_render(sd, frames: int, **params):
    """Renders `sd` under the queue schedule with extra rt_params (fold, budget, slot cap, fault injection);
    returns (image, stats)."""
    r = scenes.make_renderer(sd)
    faults = {k: params.pop(k) for k in ("ring_slots_max", "fail_alloc_above_mb") if k in params}
    if faults:
        r.set_faults(**faults)
    r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, **params)
    r.draw_frames(frames, 1000, 10)
    return r.read_image(), r.stats()


def test_default_budget_launches_of_320_frames():
    """The default colour budget on a draw whose colours exceed 8 GiB: floor(frames / 320) balanced launches of whole
    jobs (1080p x 700 frames = 17.4 GB of colours: 352 + 348 frames, 8.8 GB), bit-identical to one launch of every
    frame (a 32 GiB cap)."""
    sd = scenes.golden_scene("metal_materials", 1920, 1080)
    runs = []
    for mb in (None, 32768):
        r = scenes.make_renderer(sd)
        r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, **({"queue_budget_mb": mb} if mb else {}))
        r.draw_frames(700, 1000, 10)
        runs.append((r.read_image(), r.stats()))
    (a, sa), (b, sb) = runs
    per_frame = 240 * 135 * 64 * 12
    # (two launches with the automatic budget: two sample buffers, the second launch folds the first, rt_params.fold 3)
    assert sa.trace_launches == 2 and sa.launch_frames == 352 and sa.fold_ring == 2, sa
    assert sa.fold_bytes == 2 * 352 * per_frame, sa.fold_bytes
    assert sb.trace_launches == 1 and sb.launch_frames == 700, sb
    assert sa.queries == sb.queries
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def test_fold_allocation_failure_shrinks_the_launches():
    """Allocations the device refuses (fault injection, rt_testing_set_faults(fail_alloc_above_mb = 100): every colour-fold
    allocation above 100 MiB fails): the sample buffer (512x512 x 100 frames = 315 MB) is halved until it fits
    (launches of 25 frames); with a 160 MiB budget (under 64 frames of colours) the fold ring (4096 slots x
    32 KB) halves its budget until it fits. Both bit-identical to the default draw."""
    sd = scenes.golden_scene("metal_materials", 512, 512)
    small, st = _queue_render(sd, 100, fail_alloc_above_mb=100)
    # (four launches, each folded by the next, the last by k_accumulate: two buffers, every allocation within 100 MiB)
    assert st.fold_ring == 2 and st.launches == 5 and 0 < st.fold_bytes <= 2 * (100 << 20), st
    ring, st = _queue_render(sd, 100, fail_alloc_above_mb=100, queue_budget_mb=160)
    assert st.fold_ring == 1 and 0 < st.fold_bytes <= 100 << 20, st
    want, st = _queue_render(sd, 100)
    assert st.launches == 2 and st.fold_bytes > 100 << 20
    np.testing.assert_array_equal(small.view(np.uint32), want.view(np.uint32))
    np.testing.assert_array_equal(ring.view(np.uint32), want.view(np.uint32))


def test_fold_memory_follows_the_budget():
    """a draw through the sample buffer, then draws with a small budget (fold ring) and with the
    buffer again: each draw's colour memory is its own fold's only, within the budget (rt_stats.device_bytes,
    every device buffer the renderer holds), and the images stay bit-identical."""
    sd = scenes.config_c3(320, 192, 64)
    r = scenes.make_renderer(sd)
    r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE)
    r.draw_frames(sd.frames, 1000, 10)
    want = r.read_image()
    st = r.stats()
    base = st.device_bytes - st.fold_bytes  # image, scene, counters
    assert st.fold_ring == 0 and st.fold_bytes == 64 * 40 * 24 * 64 * 12
    for budget, fold, ring in ((1, 0, 1), (0, hrt.RT_FOLD_BUFFER, 0), (64, hrt.RT_FOLD_RING, 1), (0, 0, 0)):
        r.reset_frame_count()
        r.set_params(queue_budget_mb=budget or 32768, fold=fold)
        r.draw_frames(sd.frames, 1000, 10)
        np.testing.assert_array_equal(r.read_image().view(np.uint32), want.view(np.uint32))
        st = r.stats()
        assert st.fold_ring == ring, (budget, fold)
        assert st.device_bytes - base <= max(st.fold_bytes, 1) + (1 << 20), (budget, fold, st.device_bytes, base)
        if budget:
            assert st.fold_bytes <= (budget << 20) + (1 << 20), (budget, st.fold_bytes)


def test_renderer_calls_from_another_thread():
    """The device is bound per call (the renderer's, whatever the calling thread has current): a renderer
    created here is drawn, read and destroyed from a second host thread, bit-identical."""
    import threading
    sd = scenes.golden_scene("shadow_rendering", 64, 48)
    sd.frames = 4
    a = scenes.make_renderer(sd)
    a.draw_frames(sd.frames, 1000, 10)
    want = a.read_image()
    b = scenes.make_renderer(sd)
    out = {}

    def work():
        try:
            b.draw_frames(sd.frames, 1000, 10)
            out["img"] = b.read_image()
            out["kernel"] = b.stats().kernel
            b.close()
        except Exception as e:  # noqa: BLE001
            out["err"] = e

    t = threading.Thread(target=work)
    t.start()
    t.join(60)
    assert "err" not in out, out.get("err")
    np.testing.assert_array_equal(out["img"].view(np.uint32), want.view(np.uint32))
    assert out["kernel"] == a.stats().kernel


@pytest.mark.parametrize("budget_mb", [0, 1])
def test_release_scratch_then_draw_again(budget_mb):
    """rt_release_scratch frees the colour-fold memory (sample buffer, or the fold ring with a 1 MiB budget);
    the next draw allocates it again and renders the same bits."""
    sd = scenes.config_c3(160, 96, 64)
    r = scenes.make_renderer(sd)
    r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, **({"queue_budget_mb": budget_mb} if budget_mb else {}))
    r.draw_frames(sd.frames, 1000, 10)
    first = r.read_image()
    assert r.stats().fold_bytes > 0 and r.stats().fold_ring == (1 if budget_mb else 0)
    r.release_scratch()
    r.reset_frame_count()
    r.draw_frames(sd.frames, 1000, 10)
    np.testing.assert_array_equal(r.read_image().view(np.uint32), first.view(np.uint32))
    r.release_scratch()
    r.release_scratch()  # idempotent


@pytest.mark.parametrize("slots", [1, 2, 8])
def test_fold_ring_slot_reuse_bit_identical(slots):
    """Very few fold-ring slots (rt_testing_set_faults ring_slots_max): nearly every job waits in the free queue for a slot
    to be returned (1 slot: one job at a time). C3 (k_trace_split) and C4 (k_trace_split_tris) at 160x96,
    64 frames (two jobs per tile), and C2 (k_trace, four): images bit-identical to the tiles schedule, same
    ray counts."""
    for sd in (scenes.config_c3(160, 96, 64), scenes.config_c4(160, 96, 64), scenes.config_c2(160, 96, 64)):
        img, st = _queue_render(sd, 64, ring_slots_max=slots, queue_budget_mb=1)
        assert st.fold_ring == 1 and st.launches == 1 and st.fold_bytes <= slots * (32 << 10) + (16 << 10), st
        r = scenes.make_renderer(sd)
        r.set_params(schedule=hrt.RT_SCHEDULE_TILES)
        r.draw_frames(64, 1000, 10)
        np.testing.assert_array_equal(img.view(np.uint32), r.read_image().view(np.uint32), err_msg=sd.name)
        assert st.queries == r.stats().queries, sd.name


def test_query_count_matches_oracle():
    sd = scenes.golden_scene("dielectric_materials", 64, 48)
    r = scenes.make_renderer(sd)
    r.draw_frames(10, 1000, 10)
    img = r.read_image()
    st = r.stats()
    ref, q = scenes.oracle_render(sd, frames=10)
    assert_parity(img, ref, "dielectric 64x48")
    assert st.queries == q
    assert st.samples == 64 * 48 * 10


def test_row_partition_matches_full_image():
    sd = scenes.golden_scene("depth_of_field", 80, 50)
    full = scenes.make_renderer(sd)
    full.draw_frames(6, 1000, 10)
    fimg = full.read_image()
    for row0, step in [(0, 2), (1, 2), (2, 3), (7, 8)]:
        r = scenes.make_renderer(sd)
        r.set_params(row0=row0, row_step=step)
        r.draw_frames(6, 1000, 10)
        np.testing.assert_array_equal(r.read_image().view(np.uint32), fimg[row0::step].view(np.uint32))
    # tile-aligned row blocks dealt round-robin (the multi-GPU split of bench.py), under both schedules and
    # both colour folds; a ragged last block (50 rows) and a block that is not a multiple of the tile height
    from hrt.parallel import owned_rows
    for row0, step, block, sched, budget in [(8, 3, 8, 2, 0), (16, 3, 8, 1, 0), (0, 2, 8, 2, 1), (5, 2, 3, 2, 0),
                                             (40, 2, 8, 0, 0)]:
        r = scenes.make_renderer(sd)
        r.set_params(row0=row0, row_step=step, row_block=block, schedule=sched,
                     **({"queue_budget_mb": budget} if budget else {}))
        assert r.local_rows == len(owned_rows(row0, step, sd.height, block))
        r.draw_frames(6, 1000, 10)
        rows = owned_rows(row0, step, sd.height, block)
        np.testing.assert_array_equal(r.read_image().view(np.uint32), fimg[rows].view(np.uint32))


def test_ranks_beyond_the_image_own_no_rows():
    """with 8-row blocks dealt round-robin, a rank whose first block starts at or below the image's last
    row owns no rows (20 rows over 4 ranks: rank 3 starts at row 24). Its renderer accepts the partition, its draws
    trace nothing and its image is empty; the ranks' bands still reassemble to the full image. A resize that leaves
    a renderer without rows keeps its partition (it used to reset row0 to 0 and render rank 0's rows), and growing
    the image back gives it its blocks again."""
    from hrt.parallel import assemble, max_rows, owned_rows, rank_params
    import torch
    sd = scenes.config_c3(48, 20, 4)
    full = scenes.make_renderer(sd)
    full.draw_frames(sd.frames, 1000, 10)
    fimg = full.read_image()
    world, parts, rays = 4, [], 0
    for rank in range(world):
        for sched in (hrt.RT_SCHEDULE_QUEUE, hrt.RT_SCHEDULE_TILES):
            r = scenes.make_renderer(sd)
            r.set_params(schedule=sched, **rank_params(rank, world, 8))
            r.draw_frames(sd.frames, 1000, 10)
            img, st = r.read_image(), r.stats()
            assert img.shape == (len(owned_rows(8 * rank, world, sd.height, 8)), sd.width, 3)
            if rank == 3:
                assert img.shape[0] == 0 and st.queries == 0 and st.local_rows == 0, (sched, st.queries)
        rays += st.queries
        band = np.zeros((max_rows(world, sd.height, 8), sd.width, 3), np.float32)
        band[: len(img)] = img
        parts.append(torch.from_numpy(band))
    got = assemble(parts, sd.height, world, block=8).numpy()
    np.testing.assert_array_equal(got.view(np.uint32), fimg.view(np.uint32))
    assert rays == full.stats().queries
    r = scenes.make_renderer(sd)
    r.set_params(row0=8, row_step=2, row_block=8)
    r.resize(sd.width, 8)  # rows 8.. are gone: no rows, partition kept
    assert r.params.row0 == 8 and r.local_rows == 0
    r.draw_frames(2, 1000, 10)
    assert r.read_image().shape == (0, sd.width, 3) and r.stats().queries == 0
    r.resize(sd.width, sd.height)
    r.draw_frames(sd.frames, 1000, 10)
    np.testing.assert_array_equal(r.read_image().view(np.uint32), fimg[owned_rows(8, 2, sd.height, 8)].view(np.uint32))


@pytest.mark.parametrize("schedule", [0, 2])
def test_resume_from_checkpoint_is_bitwise(schedule):
    sd = scenes.golden_scene("metal_materials", 64, 64)
    r = scenes.make_renderer(sd)
    r.set_params(schedule=schedule)
    r.draw_frames(8, 1000, 10)
    want = r.read_image()
    a = scenes.make_renderer(sd)
    a.set_params(schedule=schedule)
    a.draw_frames(3, 1000, 10)
    ck, fc = a.read_image(), a.frame_count
    b = scenes.make_renderer(sd)
    b.set_params(schedule=schedule)
    b.write_image(ck)
    b.set_frame_count(fc)
    b.draw_frames(5, 1030, 10)
    np.testing.assert_array_equal(b.read_image().view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("schedule", [0, 2])
def test_ema_cap_and_bounce_params(schedule):
    sd = scenes.golden_scene("shadow_rendering", 48, 40)
    r = scenes.make_renderer(sd)
    r.set_params(ema_cap=3, bounces=2, schedule=schedule)
    r.draw_frames(7, 500, 7)
    ref, q = scenes.oracle_render(sd, frames=7, time0=500, dtime=7, ema_cap=3, bounces=2)
    assert_parity(r.read_image(), ref, "ema_cap=3 bounces=2")
    assert r.stats().queries == q


@pytest.mark.parametrize("schedule", [0, 2])
def test_zero_bounces_is_sky_only(schedule):
    sd = scenes.golden_scene("lambertian_materials", 32, 32)
    r = scenes.make_renderer(sd)
    r.set_params(bounces=0, schedule=schedule)
    r.draw_frames(2, 1000, 10)
    ref, q = scenes.oracle_render(sd, frames=2, bounces=0)
    assert q == 0 and r.stats().queries == 0
    assert_parity(r.read_image(), ref, "bounces=0")


@pytest.mark.parametrize("schedule", [0, 2])
def test_empty_sphere_scene_and_reset(schedule):
    sd = scenes.golden_scene("lambertian_materials", 40, 30)
    sd.spheres = hrt.spheres_array([])
    r = scenes.make_renderer(sd)
    r.set_params(schedule=schedule)
    r.draw_frames(3, 1000, 10)
    ref, _ = scenes.oracle_render(sd, frames=3)
    assert_parity(r.read_image(), ref, "empty scene (100 zero slots)")
    r.reset_frame_count()
    assert r.frame_count == 0 and not r.read_image().any()


def test_rtiow_cover_scene_small():
    sd = scenes.config_c3(160, 90, 6)
    r = scenes.make_renderer(sd)
    r.draw_frames(sd.frames, 1000, 10)
    ref, q = scenes.oracle_render(sd)
    assert_parity(r.read_image(), ref, "C3 160x90x6")
    assert r.stats().queries == q


@pytest.mark.parametrize("schedule", [1, 2])
@pytest.mark.parametrize("variant", [1, 3, 4])
def test_scan_variants_bit_identical(variant, schedule):
    """Every sphere-scan kernel variant, under both schedules, gives the oracle's bits and ray counts."""
    for sd in (scenes.config_c3(192, 108, 4), scenes.golden_scene("dielectric_materials", 128, 128),
               scenes.golden_scene("complex_scene", 128, 128)):
        sd.frames = 4
        r = scenes.make_renderer(sd)
        r.set_params(variant=variant, schedule=schedule)
        r.draw_frames(sd.frames, 1000, 10)
        ref, q = scenes.oracle_render(sd)
        assert_parity(r.read_image(), ref, f"{sd.name} variant {variant} schedule {schedule}")
        assert r.stats().variant == variant and r.stats().schedule == schedule
        assert r.stats().queries == q


@pytest.mark.parametrize("suspend_below", [1, 24, 48, 64])
def test_suspendable_walks_bit_identical(suspend_below):
    """k_trace_split (walks suspended below `suspend_below` walking lanes, finished lanes refilled) gives the
    oracle's bits and ray counts; also with the 0-bounce cap and a ragged image (partial 8x8 tiles). Its
    box/sphere test counts may differ from k_trace's (parked leaves are tested later, against a larger
    best t), never its results."""
    for sd in (scenes.config_c3(190, 106, 5), scenes.golden_scene("dielectric_materials", 128, 128),
               scenes.golden_scene("complex_scene", 100, 70)):
        sd.frames = 5
        if sd.name.startswith("complex"):
            sd.min_sphere_slots = 0
            sd.spheres = np.concatenate([sd.spheres] * 8)  # >= 32 slots: the culling BVH runs
        counts = []
        for sb in (0, suspend_below):
            r = scenes.make_renderer(sd)
            r.set_params(variant=4, schedule=2, suspend_below=sb)
            r.draw_frames(sd.frames, 1000, 10)
            st = r.stats()
            counts.append((st.queries, st.box_tests, st.sphere_tests))
            img = r.read_image()
        ref, q = scenes.oracle_render(sd)
        assert_parity(img, ref, f"{sd.name} suspend_below {suspend_below}")
        assert counts[0][0] == counts[1][0] == q
    sd = scenes.config_c3(64, 40, 3)
    sd.bounces = 0
    r = scenes.make_renderer(sd)
    r.set_params(variant=4, schedule=2, suspend_below=suspend_below)
    r.draw_frames(sd.frames, 1000, 10)
    ref, q = scenes.oracle_render(sd)
    assert_parity(r.read_image(), ref, "C3 0 bounces")
    assert r.stats().queries == q == 0


@pytest.mark.parametrize("variant", [1, 3, 4])
def test_suspendable_heap_walk_bit_identical(variant):
    """k_trace_split_tris (mixed program: sphere scan `variant`, then the reference heap walk, suspendable)
    gives the oracle's bits and ray counts, and k_trace's node/triangle test counts (the walk itself is
    unchanged); the triangle program on Suzanne and the dragon likewise. With variant 4 (culling BVH) the
    sphere walk finishes in the begin phase and only the heap walk suspends."""
    sd = scenes.config_c4(96, 72, 4)
    if variant == 4:
        sd.spheres = np.concatenate([sd.spheres] + [scenes.rtiow_spheres()[:60]])  # >= 32 slots: culling BVH
    cases = [(sd, variant)]
    if variant == 1:  # triangle program: Suzanne, and the dragon (its walks hit the 600-step cap)
        for builder, w, h in (("new_suzane", 80, 60), ("new_dragon", 64, 48)):
            scene = getattr(hrt.SceneTris, builder)(w, h)
            cases.append((scenes.SceneDef(builder, hrt.RT_MODE_TRIS, w, h, scene.camera, bvh=scene.tris_bvh.view(),
                                          frames=4), 1))
    for sd, v in cases:
        counts = []
        for sb in (0, 1, 16, 48):
            r = scenes.make_renderer(sd)
            r.set_params(variant=v if sd.mode != hrt.RT_MODE_TRIS else 0, schedule=2, suspend_below=sb)
            r.draw_frames(sd.frames, 1000, 10)
            st = r.stats()
            assert st.suspend_below == sb
            counts.append((st.queries, st.node_tests, st.tri_tests, st.sphere_tests))
            img = r.read_image()
            if sb == 16:
                ref, q = scenes.oracle_render(sd)
                assert_parity(img, ref, f"{sd.name} variant {v} suspend_below {sb}")
                assert st.queries == q
        assert all(c == counts[0] for c in counts), counts


@pytest.mark.parametrize("jf", [4, 8, 32])
def test_tail_split_bit_identical(jf):
    """The launch's last jobs dealt in parts (rt_params.tail_split 0 auto / 2 quarters / 3 eighths: the suspendable-walk
    kernels, k_trace_split and k_trace_split_tris, with the sample buffer when job_frames is a multiple of the part
    count and divides the launch's frames): images and every work count equal the draw without the split (1) and the
    oracle; the sphere program with suspend_below 0 included."""
    for sd, extra in ((scenes.config_c3(136, 80, 32), {}), (scenes.config_c3(136, 80, 32), {"suspend_below": 0}),
                      (scenes.config_c4(120, 72, 32), {}), (scenes.config_c5(96, 64, 32), {})):
        runs = []
        for tail in (1, 0, 2, 3):
            r = scenes.make_renderer(sd)
            r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, tail_split=tail, job_frames=jf, steal=1, **extra)
            r.draw_frames(sd.frames, 1000, 10)
            st = r.stats()
            runs.append((r.read_image(), (st.queries, st.node_tests, st.tri_tests, st.sphere_tests, st.box_tests)))
        for img, counts in runs[1:]:
            np.testing.assert_array_equal(runs[0][0].view(np.uint32), img.view(np.uint32), err_msg=sd.name)
            assert runs[0][1] == counts, (sd.name, runs[0][1], counts)
    ref, q = scenes.oracle_render(sd)
    assert_parity(runs[0][0], ref, f"{sd.name} tail split, job_frames {jf}")
    assert runs[0][1][0] == q


def test_count_tests_off_bit_identical():
    """rt_params.count_tests 0 (the library default; the test helper turns it on): the sphere program's k_trace_split
    without its box / sphere test counters renders the same bits and queries, reports no box / sphere tests, and the
    other kernels count as before."""
    for sd in (scenes.config_c3(136, 80, 32), scenes.config_c5(96, 64, 16)):
        runs = []
        for ct in (1, 0):
            r = scenes.make_renderer(sd)
            r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, count_tests=ct)
            r.draw_frames(sd.frames, 1000, 10)
            st = r.stats()
            runs.append((r.read_image(), st))
        (a, sa), (b, sb) = runs
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32), err_msg=sd.name)
        assert sa.queries == sb.queries and sa.box_tests > 0 and sa.sphere_tests > 0
        if sd.mode == hrt.RT_MODE_SPHERE:
            # k_trace_split<LNODES, STEAL, COUNT, PACKET>: the uncounted instantiation
            assert sb.box_tests == 0 and sb.sphere_tests == 0, sb.kernel
            assert sb.kernel.decode().split("<")[1].split(", ")[2] == "false", sb.kernel
        else:
            assert (sb.box_tests, sb.sphere_tests, sb.node_tests, sb.tri_tests) == \
                (sa.box_tests, sa.sphere_tests, sa.node_tests, sa.tri_tests)


def test_heap_top_configs_bit_identical():
    """The heap's top in LDS (rt_params.heap_lds: 1 none, 2 on = nodes 1..1023, sign-ordered, with 768-lane
    workgroups, 0 auto = on): the triangle program (Suzanne, the dragon with its capped walks), the mixed program with the linear and the
    culling-BVH sphere scans; images and ray / node / triangle counts equal across the configurations, with and
    without work stealing, and the oracle's. (The 8- and 9-level tops of round 3 were retired.)"""
    cases = [scenes.config_c4(120, 72, 5)]
    mixed = scenes.config_c4(96, 64, 4)
    mixed.spheres = np.concatenate([mixed.spheres] + [scenes.rtiow_spheres()[:60]])  # culling BVH sphere scan
    cases.append(mixed)
    for builder, w, h in (("new_suzane", 80, 60), ("new_dragon", 64, 48)):
        scene = getattr(hrt.SceneTris, builder)(w, h)
        cases.append(scenes.SceneDef(builder, hrt.RT_MODE_TRIS, w, h, scene.camera, bvh=scene.tris_bvh.view(), frames=4))
    for sd in cases:
        runs = []
        for heap_lds, steal in ((1, 1), (2, 1), (1, 2), (2, 2), (0, 0)):
            r = scenes.make_renderer(sd)
            r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, heap_lds=heap_lds, steal=steal)
            r.draw_frames(sd.frames, 1000, 10)
            st = r.stats()
            runs.append((r.read_image(), (st.queries, st.node_tests, st.tri_tests, st.sphere_tests), st.kernel.decode()))
        kernels = {k for _, _, k in runs}
        assert len(kernels) >= 4, kernels  # every configuration ran its own instantiation
        for img, counts, k in runs[1:]:
            np.testing.assert_array_equal(runs[0][0].view(np.uint32), img.view(np.uint32), err_msg=f"{sd.name} {k}")
            assert counts == runs[0][1], (sd.name, k, counts, runs[0][1])
        ref, q = scenes.oracle_render(sd)
        assert_parity(runs[-1][0], ref, f"{sd.name} heap top (auto)")
        assert runs[-1][1][0] == q


@pytest.mark.parametrize("jf", [0, 1, 3])
def test_work_stealing_bit_identical(jf):
    """Frame-block work stealing (rt_params.steal = 2; auto turns it on for short launches): waves that find the job
    queue drained claim single frames of other waves' jobs. Images and ray / node / triangle counts equal the
    draw without stealing and the oracle, for the sphere program (k_trace_split), the triangle and mixed programs
    (k_trace_split_tris, heap top in LDS or not), ragged jobs (job_frames 1 and 3 of 7 frames) and a row block."""
    cases = [(scenes.config_c3(136, 80, 7), {}), (scenes.config_c4(120, 72, 7), {}),
             (scenes.config_c4(120, 72, 7), {"heap_lds": 1}), (scenes.config_c3(136, 80, 7), {"row0": 8, "row_step": 2, "row_block": 8})]
    for sd, extra in cases:
        runs = []
        for steal in (2, 1):
            r = scenes.make_renderer(sd)
            r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, steal=steal, job_frames=jf, **extra)
            r.draw_frames(sd.frames, 1000, 10)
            st = r.stats()
            assert st.fold_ring == 0 and st.suspend_below > 0
            runs.append((r.read_image(), (st.queries, st.node_tests, st.tri_tests, st.sphere_tests, st.box_tests)))
        np.testing.assert_array_equal(runs[0][0].view(np.uint32), runs[1][0].view(np.uint32), err_msg=sd.name)
        assert runs[0][1] == runs[1][1], (sd.name, runs[0][1], runs[1][1])
        if not extra:
            ref, q = scenes.oracle_render(sd)
            assert_parity(runs[0][0], ref, f"{sd.name} stealing, job_frames {jf}")
            assert runs[0][1][0] == q


@pytest.mark.parametrize("steal,co", [(1, 3), (2, 3), (1, 2), (1, 0), (2, 0)])
def test_cost_order_bit_identical(steal, co):
    """Cost-ordered dealing (rt_params.cost_order: 2 on, learning once; 3 on, learning in every launch; 0 auto = on for
    a row partition's share and the suspendable-walk kernels, when not stealing): a launch deals the most expensive half
    of its tiles first (learnt from
    a launch's per-pixel query counts), then the rest. A renderer's first draw deals its first launch in raster order
    and the later launches in cost order, its second draw every launch in cost order; both give the images and ray /
    node / triangle counts of raster-order draws (cost_order 1) and of the oracle — sphere program (k_trace_split),
    mixed program (k_trace_split_tris, with the culling-BVH sphere walk too), the linear scan (k_trace), with stealing
    on or off, tail parts, several launches per draw and a row block."""
    budget = lambda sd: max(1, (sd.width + 7) // 8 * ((sd.height + 7) // 8) * 64 * 12 * 7 >> 20)  # noqa: E731
    cases = [(scenes.config_c3(136, 80, 21), {}), (scenes.config_c4(120, 72, 16), {}),
             (scenes.config_c5(128, 72, 16), {}), (scenes.config_c2(96, 64, 16), {"variant": 1}),
             (scenes.config_c3(136, 80, 14), {"row0": 8, "row_step": 2, "row_block": 8}),
             (scenes.config_c4(120, 72, 32), {"job_frames": 8, "tail_split": 2}),
             (scenes.config_c2(96, 64, 16), {"variant": 1, "row0": 0, "row_step": 3, "row_block": 8})]
    for sd, extra in cases:
        base = dict(schedule=hrt.RT_SCHEDULE_QUEUE, fold=hrt.RT_FOLD_BUFFER, steal=steal, **extra)
        r0 = scenes.make_renderer(sd)
        r0.set_params(cost_order=1, **base)
        r0.draw_frames(sd.frames, 1000, 10)
        s0 = r0.stats()
        want = (r0.read_image(), (s0.queries, s0.node_tests, s0.tri_tests, s0.sphere_tests, s0.box_tests))
        assert s0.ordered_launches == 0
        r = scenes.make_renderer(sd)
        # small colour budget: launches of ~7 frames, so the first draw already has ordered launches
        r.set_params(cost_order=co, queue_budget_mb=budget(sd) if sd.frames > 16 else 0, **base)
        split = extra.get("variant") != 1  # (variant 1: the linear scan's k_trace, which never steals)
        on = co >= 2 or ((steal == 1 or not split) and (extra.get("row_step", 1) > 1 or split))
        for k in range(2):
            r.reset_frame_count()
            r.draw_frames(sd.frames, 1000, 10)
            st = r.stats()
            want_ordered = (st.trace_launches - (1 if k == 0 else 0)) if on else 0
            assert st.ordered_launches == want_ordered, (sd.name, extra, k, st.ordered_launches, st.trace_launches)
            got = (r.read_image(), (st.queries, st.node_tests, st.tri_tests, st.sphere_tests, st.box_tests))
            np.testing.assert_array_equal(want[0].view(np.uint32), got[0].view(np.uint32), err_msg=f"{sd.name} draw {k}")
            assert want[1] == got[1], (sd.name, k, want[1], got[1])
        if not extra and (steal, co) == (1, 3):
            ref, q = scenes.oracle_render(sd)
            assert_parity(want[0], ref, f"{sd.name} cost order")
            assert want[1][0] == q


def test_full_size_headline_configs_agree():
    """BASELINE sizes (C3 and C4 at 1920x1080, 8 frames; the bench renders 1024 / 512): the default
    suspendable-walk kernels, plain k_trace and the tiles schedule give the same image bits and ray counts;
    the 8-way partition of bench.py (8-row blocks dealt round-robin) reassembles to the full image with the
    same total ray count; and every 90th row matches the CPU oracle bit for bit."""
    from hrt.parallel import assemble, rank_params
    for sd in (scenes.config_c3(1920, 1080, 8), scenes.config_c4(1920, 1080, 8)):
        runs = []
        for params in ({}, {"suspend_below": 0}, {"schedule": hrt.RT_SCHEDULE_TILES}):
            r = scenes.make_renderer(sd)
            r.set_params(**params)
            r.draw_frames(sd.frames, 1000, 10)
            runs.append((r.read_image(), r.stats()))
        img, st = runs[0]
        assert st.schedule == hrt.RT_SCHEDULE_QUEUE and st.suspend_below > 0
        for other, ost in runs[1:]:
            np.testing.assert_array_equal(img.view(np.uint32), other.view(np.uint32))
            assert ost.queries == st.queries
        parts, rays = [], 0
        for rank in range(8):
            r = scenes.make_renderer(sd)
            r.set_params(**rank_params(rank, 8, 8))
            r.draw_frames(sd.frames, 1000, 10)
            parts.append(torch.from_numpy(r.read_image()))
            rays += r.stats().queries
        full = assemble(parts, sd.height, 8, block=8).numpy()
        np.testing.assert_array_equal(full.view(np.uint32), img.view(np.uint32))
        assert rays == st.queries
        ref, _ = scenes.oracle_render(sd, rows=(45, 90, 12))
        assert_parity(img[45::90], ref, f"{sd.name} full size, every 90th row")


@pytest.mark.parametrize("name", sorted(scenes.oracle_fixture_cases()))
def test_hip_reproduces_oracle_fixtures(name):
    """The committed oracle outputs (tests/golden/oracle) re-rendered on the GPU through the C-ABI with the
    same row subset: image bits, ray counts and triangle-program work counts, under the auto schedule and
    the sample queue (suspendable walks), folded through the sample buffer and through the fold ring."""
    sd, (row0, step) = scenes.oracle_fixture_cases()[name]
    want, man = scenes.load_oracle_fixture(name)
    for schedule, budget in ((hrt.RT_SCHEDULE_AUTO, 0), (hrt.RT_SCHEDULE_QUEUE, 0), (hrt.RT_SCHEDULE_QUEUE, 1)):
        r = scenes.make_renderer(sd)
        r.set_params(row0=row0, row_step=step, schedule=schedule, **({"queue_budget_mb": budget} if budget else {}))
        r.draw_frames(sd.frames, 1000, 10)
        assert_parity(r.read_image(), want, f"{name} schedule {schedule} budget {budget}")
        st = r.stats()
        assert st.queries == man["queries"]
        assert (st.node_tests, st.tri_tests) == (man["node_tests"], man["tri_tests"])  # heap-walk work


def test_scan_variants_agree_at_scale():
    """Packed/interval scan vs simple scan on a larger C3 render (tens of millions of rays)."""
    sd = scenes.config_c3(640, 360, 32)
    imgs = []
    for variant in (1, 3, 4):
        r = scenes.make_renderer(sd)
        r.set_params(variant=variant, schedule=1)
        r.draw_frames(sd.frames, 1000, 10)
        imgs.append((r.read_image(), r.stats().queries))
    for img, q in imgs[1:]:
        np.testing.assert_array_equal(imgs[0][0].view(np.uint32), img.view(np.uint32))
        assert imgs[0][1] == q


def _random_scene(kind: str, seed: int):
    """Adversarial sphere sets for the culling BVH (>= 32 slots): tangent grids, radius spread over
    three decades, far-from-origin coordinates, zero-radius slots, every material."""
    rng = np.random.default_rng(seed)
    o = []
    mats = [lambda c, r: hrt.Sphere.new_lambertian(c, r, hrt.Vec3(*rng.uniform(0.1, 0.9, 3))),
            lambda c, r: hrt.Sphere.new_metal(c, r, hrt.Vec3(*rng.uniform(0.3, 0.9, 3)), float(rng.uniform(0, 0.5))),
            lambda c, r: hrt.Sphere.new_dielectric(c, r, float(rng.choice([1.33, 1.5, 2.4])))]
    off = np.zeros(3)
    if kind == "tangent_grid":  # spheres touching their neighbours: ties and grazing rays
        for i in range(-4, 4):
            for j in range(-4, 4):
                o.append(mats[(i + j) % 3](hrt.Vec3(float(i), 0.5, float(j) - 5.0), 0.5))
    elif kind == "radius_spread":
        for _ in range(120):
            c = rng.uniform([-4, -1, -9], [4, 3, -2])
            o.append(mats[rng.integers(3)](hrt.Vec3(*c), float(10 ** rng.uniform(-3, 0))))
    elif kind == "far_offset":  # the whole scene (and camera) 1e4 units away from the origin
        off = np.array([1.0e4, -2.0e4, 3.0e4])
        for _ in range(64):
            c = rng.uniform([-3, -1, -8], [3, 2, -3]) + off
            o.append(mats[rng.integers(3)](hrt.Vec3(*c), float(rng.uniform(0.1, 0.6))))
    elif kind == "nested_clusters":  # the two-pass leaf: several candidates per lane in one leaf, exact ties
        for _ in range(24):
            c = rng.uniform([-3, 0, -8], [3, 2, -3])
            rad = float(rng.uniform(0.2, 0.5))
            dup = mats[rng.integers(3)](hrt.Vec3(*c), rad)
            o.append(dup)                                                  # outer sphere
            o.append(mats[rng.integers(3)](hrt.Vec3(*c), 0.7 * rad))       # concentric inner
            o.append(mats[rng.integers(3)](hrt.Vec3(*(c + [0.3 * rad, 0, 0])), 0.5 * rad))  # overlapping
            o.append(dup)                                                  # the outer one again: a t tie, higher slot
    o.append(hrt.Sphere.new_lambertian(hrt.Vec3(*(np.array([0.0, -1000.5, -5.0]) + off)), 1000.0,
                                       hrt.Vec3(0.5, 0.5, 0.5)))
    cam = hrt.Camera.new(hrt.Vec3(*(np.array([0.5, 2.0, 3.0]) + off)), hrt.Vec3(*(np.array([0.0, 0.0, -5.0]) + off)),
                         6.0, 0.1, 0.9)
    return scenes.SceneDef(kind, hrt.RT_MODE_SPHERE, 96, 64, cam, hrt.spheres_array(o), frames=6, bounces=50,
                           min_sphere_slots=0)


@pytest.mark.parametrize("schedule", [1, 2])
@pytest.mark.parametrize("kind", ["tangent_grid", "radius_spread", "far_offset", "nested_clusters"])
def test_culling_bvh_exact_on_adversarial_scenes(kind, schedule):
    """Tiles (k_render) and the sample queue (k_trace_split; nodes in LDS: these trees have < 192 nodes)."""
    sd = _random_scene(kind, 7)
    out = []
    for variant in (1, 4):
        r = scenes.make_renderer(sd)
        r.set_params(variant=variant, schedule=schedule)
        r.draw_frames(sd.frames, 1000, 10)
        out.append((r.read_image(), r.stats()))
    for (img, st), v in zip(out[1:], (4,)):
        np.testing.assert_array_equal(out[0][0].view(np.uint32), img.view(np.uint32))
        assert out[0][1].queries == st.queries
        assert st.variant == v and st.sphere_tests < out[0][1].sphere_tests
    ref, q = scenes.oracle_render(sd)
    assert_parity(out[1][0], ref, f"{kind} BVH vs oracle")


def test_culling_bvh_with_zero_radius_slots():
    """The reference's 100-slot buffer: zero-radius slots at the origin inside the BVH (r_min = 0)."""
    sd = scenes.golden_scene("complex_scene", 96, 64)
    sd.frames = 6
    out = []
    for variant in (1, 4):
        r = scenes.make_renderer(sd)  # 25 spheres + 75 zero slots = 100 slots
        r.set_params(variant=variant, schedule=1)
        r.draw_frames(sd.frames, 1000, 10)
        out.append(r.read_image())
    for img in out[1:]:
        np.testing.assert_array_equal(out[0].view(np.uint32), img.view(np.uint32))


def test_split_walk_stack_overflow_falls_back_to_the_exact_scan():
    """2^17 coincident spheres: the culling BVH degenerates to 15 levels of median splits with every box
    hit, so k_trace_split's 14-entry LDS stack overflows and those queries fall back to the exact full
    scan (more sphere tests than the tiles kernel k_render with its 24-entry stack). Every t ties, so the lowest
    slot must win: slot 0 is the only lambertian among eight materials tiled over the slots. Both kernels, and
    k_trace_split with and without suspension, give the oracle's bits."""
    base = [hrt.Sphere.new_lambertian(hrt.Vec3(0.0, 0.0, -3.0), 1.0, hrt.Vec3(0.9, 0.3, 0.2))]
    base += [hrt.Sphere.new_metal(hrt.Vec3(0.0, 0.0, -3.0), 1.0, hrt.Vec3(0.1 * k, 0.8, 0.5), 0.05 * k)
             for k in range(1, 8)]
    sph = np.tile(hrt.spheres_array(base), 1 << 14)
    cam = hrt.Camera.new(hrt.Vec3(0.0, 0.5, 1.0), hrt.Vec3(0.0, 0.0, -3.0), 4.0, 0.0, 0.9)
    sd = scenes.SceneDef("coincident", hrt.RT_MODE_SPHERE, 24, 16, cam, sph, frames=2, bounces=8,
                         min_sphere_slots=0)
    runs = {}
    for key, params in (("tiles", {"schedule": hrt.RT_SCHEDULE_TILES}), (0, {"suspend_below": 0}),
                        (24, {"suspend_below": 24})):
        r = scenes.make_renderer(sd)
        r.set_params(variant=4, **({"schedule": hrt.RT_SCHEDULE_QUEUE} | params))
        r.draw_frames(sd.frames, 1000, 10)
        runs[key] = (r.read_image(), r.stats())
    (img0, st0), (img1, st1), (imgt, stt) = runs[0], runs[24], runs["tiles"]
    assert st0.suspend_below == 0 and st1.suspend_below == 24 and st1.queries == st0.queries == stt.queries
    assert st1.sphere_tests == st0.sphere_tests  # same walk, suspended or not
    assert st1.sphere_tests > stt.sphere_tests, (st1.sphere_tests, stt.sphere_tests)  # the fallback ran
    np.testing.assert_array_equal(img0.view(np.uint32), img1.view(np.uint32))
    np.testing.assert_array_equal(imgt.view(np.uint32), img1.view(np.uint32))
    ref, q = scenes.oracle_render(sd)
    assert q == st1.queries
    assert_parity(img1, ref, "coincident spheres, stack overflow")


def test_suzanne_tris_mode_vs_oracle():
    scene = hrt.SceneTris.new_suzane(128, 96)
    scene.init()
    for i in range(8):
        scene.set_time(1000 + 10 * i)
        scene.draw()
    img = scene.renderer.read_image()
    sd = scenes.SceneDef("suzane", hrt.RT_MODE_TRIS, 128, 96, scene.camera, bvh=scene.tris_bvh.view(), frames=8)
    ref, q = scenes.oracle_render(sd)
    assert_parity(img, ref, "new_suzane tris")


@pytest.mark.parametrize("builder", ["new_dragon", "new_lucy"])
def test_large_mesh_scenes_vs_oracle(builder):
    """scene_tris.rs:67-118: 50k / 20k-triangle heaps (n = 65536 / 32768), deep walks near the 600-step cap."""
    scene = getattr(hrt.SceneTris, builder)(64, 48)
    scene.init()
    for i in range(3):
        scene.set_time(1000 + 10 * i)
        scene.draw()
    sd = scenes.SceneDef(builder, hrt.RT_MODE_TRIS, 64, 48, scene.camera, bvh=scene.tris_bvh.view(), frames=3)
    ref, q = scenes.oracle_render(sd)
    from oracle import oracle as O
    assert_parity(scene.renderer.read_image(), ref, builder)
    r = scenes.make_renderer(sd)
    r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, job_frames=1)
    r.draw_frames(3, 1000, 10)
    np.testing.assert_array_equal(r.read_image().view(np.uint32), scene.renderer.read_image().view(np.uint32))
    st = r.stats()
    assert st.queries == q and st.node_tests == O.last_counts["node_tests"] and st.tri_tests == O.last_counts["tri_tests"]


@pytest.mark.parametrize("case", ["suzane", "dragon", "c4_v1", "c4_v3", "c4_v4"])
def test_opt_in_sah_triangle_tree(case):
    """rt_params.tri_bvh = 1 (opt-in, non-parity by contract): the SAH walk has no step
    cap, and the reference walk's 600-step cap does bind on the dragon (65 of 21,401 walks at 64x48x4).
    Checked bit for bit against the oracle with the cap lifted (and, where no walk hits the cap, that is
    the reference itself), with far fewer node tests than the reference walk."""
    if case in ("suzane", "dragon"):
        scene = hrt.SceneTris.new_suzane(80, 60) if case == "suzane" else hrt.SceneTris.new_dragon(64, 48)
        sd = scenes.SceneDef(case, hrt.RT_MODE_TRIS, scene.renderer.width, scene.renderer.height, scene.camera,
                             bvh=scene.tris_bvh.view(), frames=4)
        variant = 0
    else:
        sd = scenes.config_c4(96, 54, 4)
        variant = int(case[-1])
    from oracle import oracle as O
    capped, _ = scenes.oracle_render(sd)
    ref_nodes, n_capped = O.last_counts["node_tests"], O.last_counts["capped_walks"]
    ref, q = scenes.oracle_render(sd, step_cap=0)
    assert (n_capped > 0) == (case == "dragon")
    if n_capped == 0:
        np.testing.assert_array_equal(ref.view(np.uint32), capped.view(np.uint32))
    for schedule in (hrt.RT_SCHEDULE_TILES, hrt.RT_SCHEDULE_QUEUE):
        r = scenes.make_renderer(sd)
        r.set_params(tri_bvh=1, variant=variant, schedule=schedule)
        r.draw_frames(sd.frames, 1000, 10)
        assert_parity(r.read_image(), ref, f"{case} SAH walk, schedule {schedule}")
        st = r.stats()
        assert st.queries == q and 0 < st.node_tests < ref_nodes


@pytest.mark.parametrize("builder", ["new_cube", "new_quad"])
def test_small_tris_scenes_vs_oracle(builder):
    scene = getattr(hrt.SceneTris, builder)(64, 48)
    scene.init()
    scene.renderer.draw_frames(4, 1000, 10)
    sd = scenes.SceneDef(builder, hrt.RT_MODE_TRIS, 64, 48, scene.camera, bvh=scene.tris_bvh.view(), frames=4)
    ref, _ = scenes.oracle_render(sd)
    assert_parity(scene.renderer.read_image(), ref, builder)


@pytest.mark.parametrize("k", [0, 1, 2, 3, 5, 8])
def test_tiny_heaps_leaf_pairs_vs_oracle(k):
    """Leaf-pair walk edge cases (DESIGN §4 Leaf pairs): k triangles give n = 1 (the root is leaf 0), 2, 4, 8,
    with m odd / even / = n, so the walk's last leaf body falls inside or after a pair; both schedules (tiles:
    walk_bvh, queue: the suspendable heap_run) against the oracle, with its node and triangle test counts."""
    lines, faces = [], []
    for t in range(k):  # a fan of overlapping triangles in front of the quad camera, at several depths
        a = -1.2 + 0.3 * t
        lines += [f"v {a:.3f} -0.8 {-0.2 * t:.3f}", f"v {a + 1.1:.3f} -0.6 {-0.1 * t:.3f}", f"v {a + 0.4:.3f} 0.9 0.0"]
        faces.append(f"f {3 * t + 1} {3 * t + 2} {3 * t + 3}")
    obj = ("\n".join(lines + faces) + "\n").encode()
    tree = hrt.Tree.from_mesh(hrt.Mesh.load_obj(obj, hrt.Material.new_metal(hrt.Vec3(0.6, 0.5, 0.4), 0.3)))
    tree.build()
    sizes, nodes, tris, mats = tree.view()
    assert sizes[1] == k and sizes[0] == max(1, 1 << (k - 1).bit_length()) if k else sizes == [1, 0]
    camera = hrt.Camera.new(hrt.Vec3(0.0, 0.2, 3.5), hrt.Vec3(0.0, 0.1, -3.0), 2.2, 0.0, hrt.PI * hrt.f32(0.3))
    sd = scenes.SceneDef(f"tiny{k}", hrt.RT_MODE_TRIS, 48, 32, camera, bvh=(sizes, nodes, tris, mats), frames=3)
    ref, q = scenes.oracle_render(sd)
    from oracle import oracle as O
    want = (q, O.last_counts["node_tests"], O.last_counts["tri_tests"])
    for schedule in (hrt.RT_SCHEDULE_TILES, hrt.RT_SCHEDULE_QUEUE):
        r = scenes.make_renderer(sd)
        r.set_params(schedule=schedule, job_frames=1)
        r.draw_frames(sd.frames, 1000, 10)
        assert_parity(r.read_image(), ref, f"{k} triangles, schedule {schedule}")
        st = r.stats()
        assert (st.queries, st.node_tests, st.tri_tests) == want, (schedule, want)


def test_sign_ordered_fallback_vs_oracle():
    """The heap-top kernels' reference-form fallback (rt_kernels.hip node_hit_so<.., false>): a tree with a NaN bound
    clears so_ok, so every walk tests nodes with intersect_node's min / max on the sign-ordered layout; and an inverted
    node (min > max on one axis, swapped by the host's packing). Images and node / triangle counts equal the oracle's,
    which walks the unmodified node bytes."""
    sd = scenes.config_c4(64, 40, 3)
    sizes, nodes, tris, mats = sd.bvh
    nodes = nodes.copy()
    nodes["bound_min"][5, 0] = np.float32("nan")  # NaN: minNum drops it in the reference's min / max
    mn, mx = nodes["bound_min"][9, 1].copy(), nodes["bound_max"][9, 1].copy()
    nodes["bound_min"][9, 1], nodes["bound_max"][9, 1] = mx, mn  # inverted on y
    sd.bvh = (sizes, nodes, tris, mats)
    ref, q = scenes.oracle_render(sd)
    from oracle import oracle as O
    want = (q, O.last_counts["node_tests"], O.last_counts["tri_tests"])
    for heap_lds in (0, 1):  # the sign-ordered layout (fallback form) and the plain node bytes
        r = scenes.make_renderer(sd)
        r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, heap_lds=heap_lds)
        r.draw_frames(sd.frames, 1000, 10)
        assert_parity(r.read_image(), ref, f"NaN / inverted nodes, heap_lds {heap_lds}")
        st = r.stats()
        assert (st.queries, st.node_tests, st.tri_tests) == want, (heap_lds, want)


@pytest.mark.parametrize("schedule", [1, 2])
@pytest.mark.parametrize("variant", [1, 3, 4])
def test_mixed_mode_suzanne_ground_vs_oracle(variant, schedule):
    sd = scenes.config_c4(96, 54, 4)
    ref, q = scenes.oracle_render(sd)
    from oracle import oracle as O
    r = scenes.make_renderer(sd)
    r.set_params(variant=variant, schedule=schedule)
    r.draw_frames(sd.frames, 1000, 10)
    assert_parity(r.read_image(), ref, f"C4 mixed 96x54 variant {variant} schedule {schedule}")
    st = r.stats()
    # the reference's implicit-heap walk, step for step: identical node and triangle test counts
    assert st.queries == q and st.node_tests == O.last_counts["node_tests"] and st.tri_tests == O.last_counts["tri_tests"]
    assert st.node_tests > 0 and st.tri_tests > 0 and st.variant == variant and st.schedule == schedule


def test_large_frame_count_ema_regime():
    """Frames past SAMPLE_FRAME switch the accumulation to an EMA (shader_sphere.wgsl:268)."""
    sd = scenes.golden_scene("camera_position", 16, 16)
    r = scenes.make_renderer(sd)
    r.set_frame_count(998)
    r.draw_frames(5, 123456, 977)
    ref, _ = scenes.oracle_render(sd, frames=5, frame0=998, time0=123456, dtime=977)
    assert_parity(r.read_image(), ref, "frames 998..1002")


def test_resize_and_scene_truncation():
    """Renderer::resize (renderer.rs:271-313) zeroes the image and the frame counter: rendering after a
    resize equals a fresh renderer of the new size, bit for bit. SceneSphere::write_scene_data
    (scene_sphere.rs:24-31) keeps only the first 100 objects of a longer list."""
    sd = scenes.golden_scene("metal_materials", 48, 40)
    r = scenes.make_renderer(sd)
    r.draw_frames(3, 1000, 10)
    r.resize(40, 30)
    assert r.frame_count == 0 and not r.read_image().any()
    r.draw_frames(4, 1000, 10)
    sd2 = scenes.golden_scene("metal_materials", 40, 30)
    fresh = scenes.make_renderer(sd2)
    fresh.draw_frames(4, 1000, 10)
    np.testing.assert_array_equal(r.read_image().view(np.uint32), fresh.read_image().view(np.uint32))

    scene = hrt.SceneSphere.new(32, 24)
    scene.objects.clear()
    for i in range(120):  # the last 20 would hide everything if they were drawn
        scene.objects.append(hrt.Sphere.new_lambertian(hrt.Vec3(float(i % 10) - 4.5, float(i // 10) * 0.2, -6.0),
                                                       0.3, hrt.Vec3(0.2, 0.6, 0.4)))
    scene.objects[100:] = [hrt.Sphere.new_lambertian(hrt.Vec3(0.0, 0.0, 2.0), 1.5, hrt.Vec3(1, 0, 0))] * 20
    scene.init()
    for i in range(3):
        scene.set_time(1000 + 10 * i)
        scene.draw()
    sdt = scenes.SceneDef("trunc", hrt.RT_MODE_SPHERE, 32, 24, scene.camera, hrt.spheres_array(scene.objects[:100]),
                          frames=3)
    ref, _ = scenes.oracle_render(sdt)
    assert_parity(scene.renderer.read_image(), ref, "100-sphere truncation")


def test_rendering_performance():
    """tests/rendering_tests.rs:527-578: 20 spheres on a ring + ground, 512x512, must finish in < 5 s.
    The reference times command submission only; here the draws are synchronised, and 100 frames (the
    comment's count, TEST_FRAMES is 1 in the file) through the per-frame protocol."""
    import math
    import time
    scene = hrt.SceneSphere.new(512, 512)
    scene.objects.clear()
    for i in range(20):
        angle = np.float32(i) * np.float32(math.pi) * np.float32(2.0) / np.float32(20.0)
        x, z = float(np.cos(angle) * np.float32(3.0)), float(np.float32(-5.0) + np.sin(angle) * np.float32(3.0))
        scene.objects.append(hrt.Sphere.new_lambertian(hrt.Vec3(x, 0.0, z), 0.4,
                                                       hrt.Vec3(i / 20.0, 0.5, 1.0 - i / 20.0)))
    scene.objects.append(hrt.Sphere.new_lambertian(hrt.Vec3(0.0, -100.4, -5.0), 100.0, hrt.Vec3(0.5, 0.5, 0.5)))
    scene.init()
    t0 = time.perf_counter()
    for i in range(100):
        scene.set_time(1000 + i * 10)
        scene.draw()
    scene.renderer.synchronize()
    elapsed = time.perf_counter() - t0
    assert elapsed < 5.0, f"Rendering took too long: {elapsed:.3f} s"
    assert np.isfinite(scene.renderer.read_image()).all()


def test_range_restricted_exact_math_matches_ieee():
    """The kernels' short correctly rounded sequences (hemisphere normalize, division by a shared refined
    reciprocal, sqrt without scaling; rt_device.hpp) equal the IEEE operations bit for bit on 2^30+ random
    cases each in their stated ranges; the refined reciprocal on every significand under both signs of every binade
    2^-60 .. 2^60 (242 x 2^23 cases: the enumeration is the case index, the same for every seed)."""
    import ctypes as C
    out = (C.c_uint64 * 3)()
    for seed, n in ((1, 242 << 23), (0x9E3779B9, 1 << 30)):
        hrt._lib.check(hrt.lib().rt_check_exact_math(n, seed, out), "rt_check_exact_math")
        assert list(out) == [0, 0, 0], list(out)


def test_bad_arguments_fail_loudly():
    r = hrt.Renderer(8, 8, hrt.RT_MODE_TRIS)
    with pytest.raises(hrt.RtError):  # draw before set_camera
        r.draw()
    tri = np.zeros(1, dtype=hrt.TRIANGLE_DTYPE)
    tri["material"] = 5  # no such material
    with pytest.raises(hrt.RtError):
        r.write_bvh([1, 1], np.zeros(1, dtype=hrt.NODE_DTYPE), tri, np.zeros(1, dtype=hrt.MATERIAL_DTYPE))
    with pytest.raises(hrt.RtError):  # sizes larger than the node buffer
        r.write_bvh([4, 1], np.zeros(2, dtype=hrt.NODE_DTYPE), np.zeros(1, dtype=hrt.TRIANGLE_DTYPE),
                    np.zeros(1, dtype=hrt.MATERIAL_DTYPE))
    for n in (0, 3, 6):  # Tree::build makes n a power of two (the leaf-pair walk relies on it)
        with pytest.raises(hrt.RtError):
            r.write_bvh([n, 1], np.zeros(8, dtype=hrt.NODE_DTYPE), np.zeros(1, dtype=hrt.TRIANGLE_DTYPE),
                        np.zeros(1, dtype=hrt.MATERIAL_DTYPE))
    small = np.zeros(10, dtype=np.float32)
    assert hrt.lib().rt_read_image(r._h, small.ctypes.data_as(hrt._lib._PF), small.size) == hrt._lib.RT_ERR_ARG
    for bad in ({"variant": 2}, {"variant": 9}, {"schedule": 3}, {"tri_bvh": 2}, {"row_step": 0},
                {"suspend_below": 65}):
        with pytest.raises(hrt.RtError):  # removed variants, unknown schedule / tree, empty partition,
            r.set_params(**bad)           # a suspend threshold above the wave width
    assert hrt.Renderer(8, 8, hrt.RT_MODE_SPHERE).params.suspend_below == 24  # per-program defaults
    assert hrt.Renderer(8, 8, hrt.RT_MODE_MIXED).params.suspend_below == 24
    assert r.params.suspend_below == 32
    assert r.params.job_frames == 0  # per kernel: 32 with the suspendable walks, 16 for the linear scans
