"""Benchmark: Mrays/s of the MI355X path tracer on BASELINE.json's headline workload.

Workload (BASELINE.json metric "Mrays/sec at 1920x1080x1024spp x 50-bounce"): config C3 — the RTIOW-style
random-spheres cover scene (488 spheres, seeded), 1920x1080, 1024 frames (= spp), 50-bounce cap, sphere
mode. One STEP = one full render of that image (all 1024 frames, all rows) into a zeroed accumulation
buffer, scene already resident in HBM. A "ray" is one closest-hit query (primary + every scattered ray,
terminating miss included), counted exactly by the kernel.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): the image is split into
8-row blocks dealt round-robin (rank r renders rows 8r..8r+7, 8(r+N)..8(r+N)+7, ...: whole 8x8 tile rows, so
the sample queue's tiles stay compact, and the sky-heavy top rows spread evenly), every rank renders its rows
for all frames, then one RCCL gather over xGMI assembles the full image on rank 0 (inside the timed region).
Total work is fixed as N grows -> "scaling": "strong"; `value` is the whole-job rate.

Single-GPU proxy of that split (`--emulate-ranks N`, default 8 on a one-rank run): after the timed region,
every rank's share is rendered on this GPU in turn with the same step; the predicted N-GPU step time is the
slowest share's, and `emulated_split.efficiency` = full-image time / (N x slowest share).

Prints ONE JSON line on rank 0 (contract in the task statement), plus `roofline` (FP32-VALU bound; HIP-event
time of the render kernel on the stream it runs on) and `cpu_baseline` (the CPU oracle on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for p in (ROOT, ROOT / "hello-raytracing_amd", ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak with packed FMA (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
SPHERE_TEST_FLOP = 18  # per ray-sphere test (a, 4a hoisted per query)
BOX_TEST_FLOP = 12  # per padded slab test: 6 adds + 6 multiplies
RAY_OVERHEAD_FLOP = 90  # ~40 hit reconstruction + ~50 scatter per ray
NODE_TEST_FLOP = 27  # implicit-heap slab test (3 rcp-mul pairs, mins/maxes)
TRI_TEST_FLOP = 51  # Moller-Trumbore


def golden_check():
    """The reference's golden images (tests/golden, rendering_tests.rs:134-509) rendered on the GPU with their
    protocol (512x512, 100 frames, time 1000 + 10 i), compared in render_ppm's u8 space: per-channel max and
    mean |delta| as a fraction of 255, exact-u8 fraction, and compare_ppm_images' 2 % rule. Glass scenes differ
    from the golden GPU by construction; HIP vs the CPU oracle is bit-exact (tests/)."""
    import numpy as np

    import hrt
    import scenes

    per = {}
    for name in scenes.GOLDEN_NAMES:
        sd = scenes.golden_scene(name)
        r = scenes.make_renderer(sd)
        r.draw_frames(scenes.GOLDEN_FRAMES, 1000, 10)
        img = r.read_image()
        golden = scenes.load_golden_u8(name)
        d = np.abs(scenes.to_u8(img).astype(np.int32) - golden.astype(np.int32))
        pct = hrt.compare_ppm_images(hrt.render_ppm(r), scenes.ppm_text_from_u8(golden), 2.0)
        per[name] = {"max_abs_delta": round(float(d.max()) / 255.0, 5), "mean_abs_delta": round(float(d.mean()) / 255.0, 6),
                     "exact_u8": round(float(np.mean(d == 0)), 5), "harness_pct": round(float(pct), 4)}
    non_glass = [v["max_abs_delta"] for k, v in per.items() if k not in scenes.GLASS_GOLDENS]
    return {"scenes": len(per), "harness_pass": sum(v["harness_pct"] <= 2.0 for v in per.values()),
            "max_abs_delta_non_glass": max(non_glass),
            "max_abs_delta_all": max(v["max_abs_delta"] for v in per.values()), "per_scene": per}


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_threads() -> int:
    """Threads for the CPU baseline: the box's CPU share (16 per GPU on the pool), at most the visible CPUs."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_info() -> dict:
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        import psutil

        physical = psutil.cpu_count(logical=False)
    except Exception:  # noqa: BLE001
        physical = None
    return {"cpu_model": model, "physical_cores_visible": physical, "logical_cpus_visible": os.cpu_count()}


def find_pmc(config: str, width: int, height: int, spp: int, world: int, kernel: str):
    """The committed PMC summary (scripts/pmc.sh -> profiles/rNN/*pmc_summary.json) of exactly this workload:
    same config, resolution, spp, one rank, and the same kernel symbol. None when there is no such pass."""
    key = {"config": config, "width": width, "height": height, "spp": spp, "ranks": world, "kernel": kernel}
    for f in sorted((ROOT / "profiles").glob("r*/*pmc_summary.json"), reverse=True):
        try:
            pm = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if pm.get("_key") == key:
            pm["_file"] = str(f.relative_to(ROOT))
            return pm
    return None


def pmc_view(pm):
    """Utilisation of the VALU from the PMC pass: issue busy (VALU instructions x 2 cycles per wave64
    instruction over 1024 SIMDs x the kernel's GPU cycles) and active lanes per issued VALU instruction."""
    if not pm:
        return None
    try:
        cycles = pm["GRBM_GUI_ACTIVE"] / 8.0  # GRBM counts are summed over the 8 XCDs
        busy = pm["SQ_INSTS_VALU"] * 2.0 / (1024.0 * cycles)
        lanes = pm["SQ_THREAD_CYCLES_VALU"] / pm["SQ_ACTIVE_INST_VALU"]
    except (KeyError, ZeroDivisionError):
        return {"file": pm.get("_file")}
    return {"file": pm.get("_file"), "valu_issue_busy": round(busy, 4), "active_lanes": round(lanes, 2),
            "valu_lane_util": round(busy * lanes / 64.0, 4),
            "wait_frac": round(pm.get("SQ_WAIT_ANY", 0.0) / max(pm.get("SQ_WAVE_CYCLES", 1.0), 1.0), 4),
            "salu_insts": pm.get("SQ_INSTS_SALU"), "valu_insts": pm.get("SQ_INSTS_VALU"),
            "l2_hit_rate": (round(pm["TCC_HIT_sum"] / (pm["TCC_HIT_sum"] + pm["TCC_MISS_sum"]), 4)
                            if pm.get("TCC_HIT_sum", 0.0) + pm.get("TCC_MISS_sum", 0.0) > 0 else None)}


def launcher_selftest(args) -> int:
    """CPU rehearsal of the multi-rank path without a GPU: the self-launched ranks join a gloo group, each fills
    its interleaved rows of a W x H x 3 image with their global row index, and hrt.parallel.gather_image
    assembles them on rank 0 — the code path of the real bench minus the renderer."""
    import torch
    import torch.distributed as dist

    from hrt.parallel import gather_image, image_checksum, max_rows, rank_rows

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    block = args.row_block

    def leg(H, W):
        rows = rank_rows(rank, world, H, block)
        part = torch.zeros((max_rows(world, H, block), W, 3), dtype=torch.float32)
        part[: len(rows)] = (torch.from_numpy(rows.astype("float32"))[:, None, None] * 16.0
                             + torch.arange(W, dtype=torch.float32)[None, :, None])
        t0 = time.perf_counter()
        full = gather_image(part, H, dist if world > 1 else None, rank, world, dst=0, block=block)
        gather_s = time.perf_counter() - t0
        # (no renderer, no GPU: the device fields stay -1 and the device check reports null)
        local = {"rows": len(rows), "elapsed_s": 0.0, "trace_ms": 0.0, "gather_ms": gather_s * 1e3, "queries": 0,
                 "checksum": image_checksum(part, rows, W)}
        report = rank_reports(local, world, dist if world > 1 else None, "cpu")
        ok = rank != 0 or bool(torch.equal(full[:, 0, 0], torch.arange(H, dtype=torch.float32) * 16.0))
        return report, (image_checksum(full, range(H), W) if rank == 0 else 0), ok

    # 37 rows: with 8-row blocks rank 4 of 5+ would own none; the rows carry their index and the column. Then the
    # second leg of a multi-rank bench (C5, run after the headline config) on another shape.
    report, full_sum, ok = leg(37, 5)
    report5, full_sum5, ok5 = leg(53, 7)
    if rank == 0:
        out = {"launcher_selftest": True, "n_gpus": world, "parallelism": f"rows{world}", "row_block": block,
               "verify_gather_bitwise": ok}
        out.update(multi_rank_fields(report, full_sum, 1))
        out["c5"] = {"config": {"id": "c5", "width": 7, "height": 53}, "steps": 1, "verify_gather_bitwise": ok5,
                     **multi_rank_fields(report5, full_sum5, 1)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


REPORT_KEYS = ("rows", "elapsed_s", "trace_ms", "gather_ms", "queries", "device", "pci", "torch_device", "torch_pci")


def pci_code(pci) -> int:
    """(domain, bus, device) as one integer (-1: no GPU)."""
    return -1 if pci is None else (int(pci[0]) << 16) | (int(pci[1]) << 8) | int(pci[2])


def pci_str(code: int):
    return None if code < 0 else f"{code >> 16:04x}:{(code >> 8) & 0xFF:02x}:{code & 0xFF:02x}"


def rank_reports(local: dict, world: int, dist, device) -> list:
    """Every rank's own figures (rows owned, timed-region wall time, trace kernel time, gather time, rays, image
    checksum, and the GPU it drew on: the renderer's device (rt_get_device) next to torch's current device, each as
    ordinal and PCI location), collected on every rank by one all_gather after the timed region (the
    8-GPU run is the driver's alone, so its line must say what each rank did, and where)."""
    import torch

    t = torch.tensor([float(local.get(k, -1)) for k in REPORT_KEYS], dtype=torch.float64, device=device)
    # (the checksum as a signed 64-bit word)
    c = torch.tensor([((int(local["checksum"]) + 2**63) % 2**64) - 2**63], dtype=torch.int64, device=device)
    if dist is None:
        ts, cs = [t], [c]
    else:
        ts = [torch.zeros_like(t) for _ in range(world)]
        cs = [torch.zeros_like(c) for _ in range(world)]
        dist.all_gather(ts, t)
        dist.all_gather(cs, c)
    out = []
    for k in range(world):
        v = ts[k].cpu().tolist()
        d = {"rank": k, **{key: v[i] for i, key in enumerate(REPORT_KEYS)}, "checksum": int(cs[k].cpu().item())}
        for key in ("rows", "queries", "device", "pci", "torch_device", "torch_pci"):
            d[key] = int(d[key])
        out.append(d)
    return out


def device_check(report: list, distinct: bool):
    """(ok, message): every rank's renderer draws on its torch device (same ordinal and PCI location) and, with one
    GPU per rank (nccl), no two ranks share a GPU. None when the ranks have no GPU (the CPU launcher self-test)."""
    if any(d["device"] < 0 or d["torch_device"] < 0 for d in report):
        return None, None
    bad = [d["rank"] for d in report if (d["device"], d["pci"]) != (d["torch_device"], d["torch_pci"])]
    if bad:
        return False, (f"ranks {bad}: the renderer's GPU differs from torch's current device (two HIP runtimes, or "
                       f"set_device not seen by the renderer)")
    if distinct:
        seen = {}
        for d in report:
            seen.setdefault(d["pci"], []).append(d["rank"])
        shared = {pci_str(k): v for k, v in seen.items() if len(v) > 1}
        if shared:
            return False, f"ranks share a GPU: {shared}"
    return True, None


def multi_rank_fields(report: list, full_checksum: int, steps: int, distinct_gpus: bool = True) -> dict:
    """The JSON line's per-rank block: per-rank elapsed / trace / gather times, rows and GPU (renderer and torch), the
    gather's own time, the destination rank's check that the gathered image's position-dependent checksum equals the
    sum of the ranks' local ones (hrt.parallel.image_checksum; mod 2^64), and the device check (device_check)."""
    ranks = [{"rank": d["rank"], "rows": d["rows"], "elapsed_s": round(d["elapsed_s"], 4),
              "trace_ms_per_step": round(d["trace_ms"] / steps, 3), "gather_ms_per_step": round(d["gather_ms"] / steps, 3),
              "rays_per_step": round(d["queries"] / steps),
              "device": d["device"], "pci": pci_str(d["pci"]), "torch_device": d["torch_device"],
              "torch_pci": pci_str(d["torch_pci"])} for d in report]
    total = sum(d["checksum"] for d in report)
    ok, msg = device_check(report, distinct_gpus)
    return {
        "ranks": ranks,
        "gather_ms_per_step": round(max(d["gather_ms"] for d in report) / steps, 3),
        "slowest_rank": max(report, key=lambda d: d["elapsed_s"])["rank"],
        "gather_checksum_ok": (total - int(full_checksum)) % 2**64 == 0,
        "device_check_ok": ok,
        "device_error": msg,
    }


def cpu_baseline(sd, threads: int, rows: int, frames: int):
    """The oracle (C restatement, OpenMP over rows) on a bounded sample of the same workload."""
    import scenes

    H = sd.height
    step = max(1, H // rows)
    n = len(range(0, H, step))
    t0 = time.perf_counter()
    _, q = scenes.oracle_render(sd, frames=frames, rows=(0, step, n), threads=threads)
    dt = time.perf_counter() - t0
    return {
        "value": round(q / dt / 1e6, 3),
        "unit": "Mrays/s",
        "samples_per_s": round(n * sd.width * frames / dt, 1),
        "cores": threads,
        "kind": "port",
        "algorithm": (f"linear-scan oracle: every ray tests all {len(sd.spheres)} sphere slots (the reference's "
                      "algorithm); the GPU kernel culls with a BVH, so the ratio mixes algorithm and hardware"),
        "threads": threads,
        # (why not every core) the GPU box gives one GPU's job a 16-thread CPU share (OMP_NUM_THREADS=16 on
        # the pool; the machine's other cores belong to the other GPUs' jobs), so the baseline uses that share; per core:
        "value_per_core": round(q / dt / 1e6 / threads, 3),
        "cores_note": "16 = the CPU share of one GPU on the box (the visible cores serve 8 GPUs' jobs); scale "
                      "value_per_core by a core count for other hosts",
        **cpu_info(),
        "sample": f"{sd.name}: {n} rows (every {step}th) x {sd.width} px x {frames} frames, {q} rays in {dt:.1f} s",
    }


MODE_NAMES = {0: "sphere", 1: "tris", 2: "mixed"}
# Rows per block of the multi-GPU row partition: whole 8-row tile rows, except C4, whose Suzanne rows
# spread more evenly over the ranks in 4-row blocks (8-way emulated split 0.83 -> 0.857; C3 prefers 8: 0.957 against
# 0.950 with 4; profiles/r05/rb/)
ROW_BLOCK = {"c4": 4}
# the frame protocol of every timed step (the reference's golden tests: time 1000 + 10 i, rendering_tests.rs:14-28)
TIME0, DTIME = 1000, 10


def timed_knobs(frames_per_launch: int = 1024, variant: int = 0, schedule: int = 0, tri_bvh: int = 0, **extra) -> dict:
    """rt_params of the timed draws (the library's defaults unless a flag overrides them): count_tests 0, so the sphere
    program's k_trace_split runs uncounted (its box / sphere counts come from a counting warmup draw, bit-identical).
    tests/test_gpu_timed.py renders the timed configurations through this same function."""
    return dict(frames_per_launch=frames_per_launch, variant=variant, schedule=schedule, tri_bvh=tri_bvh,
                count_tests=0, **extra)


def emulate_split(sd, knobs: dict, n: int, args, full_img, full_s: float, full_rays: float) -> dict:
    """Single-GPU proxy of the n-rank row split: every rank's share (rank_params(k, n, row_block)) rendered on
    this GPU in turn with the bench's step (reset, draw all frames, copy the image out, synchronise), warmed up
    and timed like the full image. On n GPUs the step takes the slowest share (+ the gather of <= 3 MB per
    rank for C3, ~0.1 ms over xGMI), so efficiency = full-image step / (n x slowest share). The shares are
    also put back together and compared with the full image bit for bit."""
    import numpy as np
    import torch

    import scenes
    from hrt.parallel import assemble, rank_params

    shares, parts = [], []
    for k in range(n):
        rk = scenes.make_renderer(sd)
        rk.set_params(**rank_params(k, n, args.row_block), **knobs)
        buf = torch.zeros((rk.local_rows, sd.width, 3), dtype=torch.float32, device="cuda")

        def share_step():
            rk.reset_frame_count()
            rk.draw_frames(sd.frames, TIME0, DTIME)
            rk.copy_image_to_device(buf.data_ptr(), buf.numel())
            return rk.stats()

        for _ in range(max(1, args.warmup)):
            share_step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        rays = trace_ms = 0.0
        for _ in range(args.steps):
            st = share_step()
            rays += st.queries
            trace_ms += st.trace_ms
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / args.steps
        shares.append({"rank": k, "rows": rk.local_rows, "ms_per_step": round(dt * 1e3, 3),
                       "trace_ms": round(trace_ms / args.steps, 3), "mrays_s": round(rays / args.steps / dt / 1e6, 1)})
        parts.append(buf.cpu())
        rk.close()
        del buf
        log(f"emulated rank {k}/{n}: {shares[-1]}")
    slowest = max(s["ms_per_step"] for s in shares)
    same = None
    if full_img is not None:
        whole = assemble(parts, sd.height, n, block=args.row_block)
        same = bool(torch.equal(whole.view(torch.int32), full_img.cpu().view(torch.int32)))
    return {
        "ranks": n,
        "row_block": args.row_block,
        "full_ms_per_step": round(full_s * 1e3, 3),
        "full_mrays_s": round(full_rays / full_s / 1e6, 1),
        "predicted_ms_per_step": slowest,
        "predicted_mrays_s": round(full_rays / (slowest * 1e-3) / 1e6, 1),
        "efficiency": round(full_s * 1e3 / (n * slowest), 4),
        "rank0_mrays_s": shares[0]["mrays_s"],
        "bitwise_equal_full_image": same,
        "per_rank": shares,
    }


def run_leg(sd, knobs: dict, args, dist, rank: int, world: int, dev, steps: int, warmup: int, tag: str = "") -> dict:
    """One timed leg of the bench on this rank: the renderer for this rank's rows (8-row blocks dealt round-robin),
    `warmup` counting steps, then `steps` timed steps bracketed by a barrier + synchronize on both sides. A step =
    reset, draw every frame (TIME0 + f * DTIME), copy the image into the rank's band, gather the bands on rank 0."""
    import torch

    import scenes
    from hrt.parallel import gather_image, image_checksum, max_rows, owned_rows, rank_params

    r = scenes.make_renderer(sd)
    r.set_params(**rank_params(rank, world, args.row_block), **knobs)
    local_rows = r.local_rows
    part = torch.zeros((max_rows(world, sd.height, args.row_block), sd.width, 3), dtype=torch.float32, device=dev)
    gathered = [torch.empty_like(part) for _ in range(world)] if (world > 1 and rank == 0) else None
    full = torch.empty((sd.height, sd.width, 3), dtype=torch.float32, device=dev) if rank == 0 else None

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    gather_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    gather_ms = [0.0]

    def step():
        r.reset_frame_count()
        r.draw_frames(sd.frames, TIME0, DTIME)
        r.copy_image_to_device(part.data_ptr(), local_rows * sd.width * 3)  # syncs the renderer stream
        st = r.stats()
        gather_ev[0].record()
        gather_image(part, sd.height, dist, rank, world, dst=0, gathered=gathered, out=full, block=args.row_block)
        gather_ev[1].record()
        if world > 1:
            # the gather reads `part` on the collective's stream; the next step's copy into `part` runs on the
            # renderer's own stream, which does not order against it: finish the gather first
            torch.cuda.current_stream().synchronize()
        gather_ev[1].synchronize()
        gather_ms[0] += gather_ev[0].elapsed_time(gather_ev[1])
        return st

    log(f"{tag + ' ' if tag else ''}rank {rank}/{world}: {sd.name} {sd.width}x{sd.height} x{sd.frames} frames, "
        f"{len(sd.spheres) if sd.spheres is not None else 0} spheres, {local_rows} rows, warmup {warmup}")
    counted = None  # (box tests, sphere tests) of one step, from a counting draw

    def counting_step():
        r.set_params(count_tests=1)
        st = step()
        r.set_params(count_tests=0)
        return st.box_tests, st.sphere_tests

    for i in range(warmup):
        t = time.perf_counter()
        counted = counting_step()
        torch.cuda.synchronize()
        log(f"{tag} warmup {i}: {time.perf_counter() - t:.2f} s")

    barrier()
    gather_ms[0] = 0.0
    t0 = time.perf_counter()
    L = {"queries": 0, "kernel_ms": 0.0, "launches": 0, "box_tests": 0, "sphere_tests": 0, "node_tests": 0,
         "tri_tests": 0, "variant": 0, "schedule": 0, "suspend": 0, "trace_ms": 0.0, "trace_launches": 0,
         "st_last": None}
    uncounted = False
    for i in range(steps):
        st = step()
        L["st_last"] = st
        for k in ("queries", "kernel_ms", "launches", "box_tests", "sphere_tests", "node_tests", "tri_tests",
                  "trace_ms", "trace_launches"):
            L[k] += getattr(st, k)
        uncounted = st.box_tests == 0 and st.sphere_tests == 0
        L["variant"], L["schedule"], L["suspend"] = st.variant, st.schedule, st.suspend_below
        log(f"{tag} step {i}: {st.queries / 1e9:.3f} G rays, kernels {st.kernel_ms:.1f} ms (trace {st.trace_ms:.1f}), "
            f"{st.sphere_tests / max(st.queries, 1):.1f} sphere + {st.box_tests / max(st.queries, 1):.1f} box tests/ray")
    barrier()
    L["elapsed"] = time.perf_counter() - t0
    if steps and uncounted:  # the timed kernels did not count: the per-step counts of a counting draw
        if counted is None:  # (no warmup: one more draw after the timed region, rank-local, no collective)
            r.set_params(count_tests=1)
            r.reset_frame_count()
            r.draw_frames(sd.frames, TIME0, DTIME)
            st_c = r.stats()
            r.set_params(count_tests=0)
            counted = (st_c.box_tests, st_c.sphere_tests)
        L["box_tests"], L["sphere_tests"] = counted[0] * steps, counted[1] * steps
    # this rank's report: rows, times, rays, its band's position-dependent checksum, and the GPU it drew on — the
    # renderer's (rt_get_device) next to torch's current device
    ordinal, pci = r.device()
    tdev = torch.cuda.current_device()
    tp = torch.cuda.get_device_properties(tdev)
    p = rank_params(rank, world, args.row_block)
    L["local"] = {"rows": local_rows, "elapsed_s": L["elapsed"], "trace_ms": L["trace_ms"], "gather_ms": gather_ms[0],
                  "queries": L["queries"], "device": ordinal, "pci": pci_code(pci), "torch_device": tdev,
                  "torch_pci": pci_code((tp.pci_domain_id, tp.pci_bus_id, tp.pci_device_id)),
                  "checksum": image_checksum(part, owned_rows(p["row0"], p["row_step"], sd.height, args.row_block),
                                             sd.width)}
    L.update(renderer=r, full=full, local_rows=local_rows)
    return L


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=["c1", "c2", "c3", "c4", "c5"],
                    help="BASELINE.json config (c3 = the headline metric)")
    ap.add_argument("--frames", type=int, default=None, help="spp per step (default: the config's)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--frames-per-launch", type=int, default=1024, help="tiles schedule: frames per launch")
    ap.add_argument("--schedule", type=int, default=0, help="0 auto (queue), 1 tiles, 2 sample queue")
    ap.add_argument("--job-frames", type=int, default=None, help="sample queue: frames per 8x8-tile job "
                                                                 "(default: the library's)")
    ap.add_argument("--suspend-below", type=int, default=None,
                    help="sample queue, sphere BVH: suspend a wave's walks below this many walking lanes "
                         "(default: the library's)")
    ap.add_argument("--queue-budget-mb", type=int, default=None,
                    help="sample queue: colour-buffer budget per chunk in MiB (default: the library's)")
    ap.add_argument("--fold", type=int, default=None,
                    help="sample queue colour fold: 0 auto, 1 sample buffer + k_accumulate, 2 fold ring, 3 two sample "
                         "buffers, each launch folded by the next")
    ap.add_argument("--heap-lds", type=int, default=None,
                    help="triangle / mixed programs: 0 auto (heap top in LDS when it fits), 1 off")
    ap.add_argument("--steal", type=int, default=None,
                    help="sample queue: frame-block work stealing, 0 auto (short launches), 1 off, 2 on")
    ap.add_argument("--tail-split", type=int, default=None, help="sample queue: 0 auto (quarter jobs at the end), 1 off")
    ap.add_argument("--cost-order", type=int, default=None,
                    help="sample queue: 0 auto (the most expensive tiles first for a row partition's shares "
                         "without stealing), 1 off, 2 on")
    ap.add_argument("--packet", type=int, default=None,
                    help="sphere program: primary rays walked as one packet per frame block: 0 auto (off: -8 %% on C3), 1 off, "
                         "2 on")
    ap.add_argument("--tri-bvh", type=int, default=0,
                    help="triangle program: 0 the reference heap walk (parity), 1 opt-in SAH tree (non-parity)")
    ap.add_argument("--variant", type=int, default=0,
                    help="sphere-scan kernel: 0 auto, 1 simple, 2 packed, 3 deferred, 4 culling BVH")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only to rehearse on one GPU)")
    ap.add_argument("--verify", action="store_true", help="rank 0 re-renders the image alone and compares")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-golden", action="store_true", help="skip the golden-image check (rank 0, after timing)")
    ap.add_argument("--cpu-rows", type=int, default=108)
    ap.add_argument("--cpu-frames", type=int, default=128)
    ap.add_argument("--row-block", type=int, default=None,
                    help="multi-GPU split: rows per block dealt round-robin (8 = whole 8x8 tile rows; 1 = single "
                         "interleaved rows); default ROW_BLOCK's per-workload choice")
    ap.add_argument("--emulate-ranks", type=int, default=None,
                    help="single-GPU proxy of the N-rank split: render every rank's share here in turn after the "
                         "timed region (default 8 on a one-rank run, 0 = off)")
    ap.add_argument("--c5-leg", type=int, default=None,
                    help="after the timed config, time a short C5 leg (BASELINE's 8-GPU config): default on for "
                         "multi-rank runs, 1 forces it on one rank, 0 off")
    ap.add_argument("--c5-steps", type=int, default=3)
    ap.add_argument("--c5-warmup", type=int, default=1)
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="CPU-only rehearsal of the multi-rank path (self-launch, gloo, row-tile gather): no GPU")
    args = ap.parse_args()
    args.row_block_given = args.row_block is not None  # (the C5 leg keeps its own partition unless one was given)
    if args.row_block is None:
        args.row_block = ROW_BLOCK.get(args.config, 8)

    from hrt.launch import needs_self_launch, spawn_ranks

    if needs_self_launch(args.gpus):
        # no external launcher: run this script as N ranks (torch.distributed.run) before any GPU call here
        log(f"--gpus {args.gpus} without WORLD_SIZE: launching {args.gpus} ranks on 127.0.0.1")
        return spawn_ranks(args.gpus, str(Path(__file__).resolve()), sys.argv[1:])
    if args.launcher_selftest:
        return launcher_selftest(args)

    import torch

    import hrt  # noqa: F401  (loads lib/libhrt.so)
    import scenes
    from hrt.parallel import image_checksum

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus {args.gpus}: using WORLD_SIZE")
    dist = None
    if world > 1:
        import torch.distributed as dist

        # one rank per GPU; (rehearsal only: more ranks than GPUs share devices, with --backend gloo)
        dev_index = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_index)
        if args.backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(args.backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    sd = scenes.CONFIGS[args.config]()
    if args.width or args.height or args.frames:
        sd.width = args.width or sd.width
        sd.height = args.height or sd.height
        sd.frames = args.frames or sd.frames
    nslots = len(sd.spheres)
    extra = {} if args.suspend_below is None else {"suspend_below": args.suspend_below}
    if args.job_frames is not None:
        extra["job_frames"] = args.job_frames
    if args.queue_budget_mb is not None:
        extra["queue_budget_mb"] = args.queue_budget_mb
    if args.fold is not None:
        extra["fold"] = args.fold
    if args.heap_lds is not None:
        extra["heap_lds"] = args.heap_lds
    if args.steal is not None:
        extra["steal"] = args.steal
    if args.tail_split is not None:
        extra["tail_split"] = args.tail_split
    if args.cost_order is not None:
        extra["cost_order"] = args.cost_order
    if args.packet is not None:
        extra["packet"] = args.packet
    # the timed draws run the default kernels (count_tests 0: the sphere program's k_trace_split does not count its box
    # and sphere tests); the warmup draws count them (count_tests 1) for the per-ray figures of the line, the same
    # every step (bit-identical draws)
    knobs = timed_knobs(args.frames_per_launch, args.variant, args.schedule, args.tri_bvh, **extra)
    L = run_leg(sd, knobs, args, dist, rank, world, dev, args.steps, args.warmup)
    full, local_rows, elapsed, queries = L["full"], L["local_rows"], L["elapsed"], L["queries"]
    st_last, schedule, suspend, variant = L["st_last"], L["schedule"], L["suspend"], L["variant"]
    emulated = None
    n_emul = args.emulate_ranks if args.emulate_ranks is not None else (8 if world == 1 else 0)
    if world == 1 and n_emul > 1:
        emulated = emulate_split(sd, knobs, n_emul, args, full, elapsed / args.steps, queries / args.steps)

    stats_t = torch.tensor([elapsed, float(queries), L["trace_ms"], float(L["trace_launches"]), float(L["box_tests"]),
                            float(L["sphere_tests"]), float(L["node_tests"]), float(L["tri_tests"]), L["kernel_ms"]],
                           dtype=torch.float64,
                           device=dev if args.backend == "nccl" else "cpu")
    if dist is not None:
        all_t = [torch.zeros_like(stats_t) for _ in range(world)]
        dist.all_gather(all_t, stats_t)
        all_t = torch.stack(all_t).cpu().numpy()
    else:
        all_t = stats_t.cpu().numpy()[None]
    t_max = float(all_t[:, 0].max())
    total_q = float(all_t[:, 1].sum())
    # per-rank figures, the gather's checksum check and the device check (multi-rank runs)
    report = None
    coll_dev = dev if args.backend == "nccl" else "cpu"
    if world > 1:
        report = rank_reports(L["local"], world, dist, coll_dev)
    # BASELINE.json's 8-GPU config is C5 (4K x 4096 spp, row tiles + RCCL gather): after the headline leg a multi-rank
    # run times a short C5 leg too (1 warmup + 3 steps; ~1.2 s per step on 8 ranks), same partition, same report
    c5 = None
    c5_on = args.c5_leg if args.c5_leg is not None else (world > 1 and args.config != "c5")
    if c5_on:
        # the headline leg's renderer (and its colour buffer) goes first: one leg's memory at a time
        del L["renderer"]
        torch.cuda.synchronize()
        sd5 = scenes.CONFIGS["c5"]()
        head_block = args.row_block
        args.row_block = args.row_block if args.row_block_given else ROW_BLOCK.get("c5", 8)
        L5 = run_leg(sd5, timed_knobs(args.frames_per_launch, 0, 0, 0), args, dist, rank, world, dev, args.c5_steps,
                     args.c5_warmup, tag="c5")
        rep5 = rank_reports(L5["local"], world, dist, coll_dev)
        c5 = {"L": L5, "report": rep5, "sd": sd5, "row_block": args.row_block}
        del L5["renderer"]
        args.row_block = head_block

    device_error = None
    if rank == 0:
        value = total_q / t_max / 1e6
        # roofline of the ray-tracing kernel (k_trace under the sample queue, k_render under tiles) on
        # rank 0: algorithmic FLOPs per launch / its HIP-event launch time (events around each launch).
        # Algorithmic = SURVEY 8(d)'s per-ray figure (18 FLOP per slot + ~90 for hit record and scatter)
        # x rays. executed = the tests the kernel actually ran (exact counters): 18 per ray-sphere test,
        # 12 per padded box test — with the culling BVH the two differ by ~30x.
        my_q, my_ms, my_launches = float(all_t[0, 1]), float(all_t[0, 2]), float(all_t[0, 3])
        my_box, my_sph = float(all_t[0, 4]), float(all_t[0, 5])
        my_nodes, my_tris = float(all_t[0, 6]), float(all_t[0, 7])
        nl = max(my_launches, 1.0)
        avg_launch_ms = my_ms / nl
        # the triangle program runs the reference's own walk: its node/triangle tests are algorithmic as is
        tri_flop = NODE_TEST_FLOP * my_nodes + TRI_TEST_FLOP * my_tris
        flop_per_launch = ((SPHERE_TEST_FLOP * nslots + RAY_OVERHEAD_FLOP) * my_q + tri_flop) / nl
        achieved = flop_per_launch / (avg_launch_ms * 1e-3) / 1e12
        executed_flop_per_launch = (SPHERE_TEST_FLOP * my_sph + BOX_TEST_FLOP * my_box + RAY_OVERHEAD_FLOP * my_q
                                    + tri_flop) / nl
        executed = executed_flop_per_launch / (avg_launch_ms * 1e-3) / 1e12
        px = local_rows * sd.width
        if schedule == 2:  # one colour per sample (12 B; 16 B through the fold ring); the spheres read once
            per_sample = 16.0 if st_last.fold_ring == 1 else 12.0
            # (fold 3: launches 2..n also read the launch before's colours, 12 B per sample, and fold them into the
            # image: on average (n - 1) / n of a launch's colours more per trace launch)
            tl = max(int(st_last.trace_launches), 1)
            if st_last.fold_ring == 2:
                per_sample += 12.0 * (tl - 1) / tl
            alg_bytes = per_sample * px * sd.frames * args.steps / nl + 64.0 * nslots  # + ragged-tile padding
        else:  # k_render reads and writes the framebuffer once per launch
            alg_bytes = 24.0 * px + 64.0 * nslots
        kernel_sym = st_last.kernel.decode() if st_last is not None else ""
        pmc = find_pmc(args.config, sd.width, sd.height, sd.frames, world, kernel_sym)
        traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
        executed_tflops = executed
        out = {
            "metric": ("Mrays/sec at 1920x1080x1024spp x 50-bounce (RTIOW cover scene)"
                       if args.config == "c3" and (sd.width, sd.height, sd.frames) == (1920, 1080, 1024)
                       else f"Mrays/sec, {sd.name} {sd.width}x{sd.height}x{sd.frames}spp x {sd.bounces}-bounce"),
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 2),
            # SURVEY 8(d) / BASELINE.md 3: pixel-samples per second (W x H x spp per step)
            "samples_per_s": round(sd.width * sd.height * sd.frames * args.steps / t_max, 1),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded RTIOW-style scene, committed generator tests/scenes.py)",
            "config": {
                "workload": sd.name,
                "id": args.config,
                "width": sd.width,
                "height": sd.height,
                "spp": sd.frames,
                "bounces": sd.bounces,
                "spheres": nslots,
                "rays_per_step": round(total_q / args.steps),
                "rays_per_sample": round(total_q / args.steps / (sd.width * sd.height * sd.frames), 4),
                "parallelism": f"rows{world}",
                "row_block": args.row_block,
                # how the sample queue folded the colours in frame order (rt_params.queue_budget_mb, fold):
                # "sample-buffer" (+ k_accumulate), "sample-buffers-folded-by-next-launch" (two buffers, each launch
                # folds the one before, k_accumulate the last) or the bounded-memory "fold-ring"; device bytes it used
                "fold": (["sample-buffer", "fold-ring", "sample-buffers-folded-by-next-launch"][st_last.fold_ring]
                         if schedule == 2 else "in-register"),
                "fold_bytes": int(st_last.fold_bytes) if schedule == 2 else 0,
                # frames per trace launch (the sample buffer's balanced launches, rt_params.queue_budget_mb)
                "launch_frames": int(st_last.launch_frames) if schedule == 2 else 0,
                # trace launches of the last timed step that dealt their tiles in learnt cost order (rt_params.cost_order)
                "ordered_launches": int(st_last.ordered_launches) if schedule == 2 else 0,
                # the timed steps redraw the warmup's scene: tile costs learnt before the timed region (a cold single
                # render runs 1 learning + 2 ordered launches for C3, ~0.6 % slower)
                "warm": bool(args.warmup > 0 and schedule == 2 and st_last.ordered_launches > 0),
            },
            # The path is FP32-VALU issue bound (no MFMA: no dense contraction; HBM ~2 % busy). `achieved` =
            # the FP32 FLOPs the kernel executes (its exact in-kernel test counters x FLOP per test, + the
            # per-ray hit record / scatter) / the HIP-event time of its launches on the renderer's stream.
            "roofline": {
                "bound": "fp32-valu",
                "achieved": round(executed_tflops, 3),
                "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(executed_tflops / FP32_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "kernel": kernel_sym,
                "schedule": {1: "tiles", 2: "sample-queue"}.get(schedule, str(schedule)),
                "suspend_below": suspend,
                "sphere_variant": variant,
                "avg_launch_ms": round(avg_launch_ms, 3),
                "launches_per_step": round(nl / args.steps, 3),
                "all_kernels_ms_per_step": round(float(all_t[0, 8]) / args.steps, 3),
                "flop_model": {"sphere_test": SPHERE_TEST_FLOP, "box_test": BOX_TEST_FLOP, "per_ray": RAY_OVERHEAD_FLOP,
                               "heap_node_test": NODE_TEST_FLOP, "tri_test": TRI_TEST_FLOP},
                "sphere_tests_per_ray": round(my_sph / max(my_q, 1.0), 3),
                "box_tests_per_ray": round(my_box / max(my_q, 1.0), 3),
                "tri_node_tests_per_ray": round(my_nodes / max(my_q, 1.0), 3),
                "tri_tests_per_ray": round(my_tris / max(my_q, 1.0), 3),
                "executed_flop_per_launch": executed_flop_per_launch,
                # SURVEY 8(d)'s per-ray price of the reference algorithm (a linear scan over every slot): the
                # culling BVH delivers that work ~24x faster than it could be executed literally, so this
                # ratio exceeds 1 and is not a utilisation
                "linear_scan_equiv_tflops": round(achieved, 3),
                "linear_scan_equiv_frac": round(achieved / FP32_PEAK_TFLOPS, 4),
                "alg_hbm_bytes_per_launch": alg_bytes,
                "hbm_gbs_alg": round(alg_bytes / (avg_launch_ms * 1e-3) / 1e9, 3),
                # HBM view (north star): the committed PMC pass of this exact config and kernel, per launch
                "hbm_gbs_traffic": (round(traffic / (avg_launch_ms * 1e-3) / 1e9, 3) if traffic else None),
                "hbm_frac": (round(traffic / (avg_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if traffic else None),
                "pmc": pmc_view(pmc),
            },
        }
        # one GPU per rank under RCCL: no two ranks may share one (a gloo rehearsal on one GPU shares it by design)
        distinct = args.backend == "nccl"
        device_error = None
        if report is not None:
            out.update(multi_rank_fields(report, image_checksum(full, range(sd.height), sd.width), args.steps, distinct))
            device_error = out["device_error"]
        if c5 is not None:
            L5, rep5, sd5 = c5["L"], c5["report"], c5["sd"]
            t5 = max(d["elapsed_s"] for d in rep5)
            q5 = sum(d["queries"] for d in rep5)
            st5 = L5["st_last"]
            blk = {
                "metric": f"Mrays/sec, {sd5.name} {sd5.width}x{sd5.height}x{sd5.frames}spp x {sd5.bounces}-bounce",
                "value": round(q5 / t5 / 1e6, 2),
                "unit": "Mrays/s",
                "steps": args.c5_steps,
                "warmup": args.c5_warmup,
                "ms_per_step": round(t5 / max(args.c5_steps, 1) * 1e3, 2),
                "config": {"workload": sd5.name, "id": "c5", "width": sd5.width, "height": sd5.height, "spp": sd5.frames,
                           "bounces": sd5.bounces, "spheres": len(sd5.spheres), "parallelism": f"rows{world}",
                           "row_block": c5["row_block"], "rays_per_step": round(q5 / max(args.c5_steps, 1)),
                           "kernel": st5.kernel.decode() if st5 is not None else "",
                           "launch_frames": int(st5.launch_frames) if st5 is not None else 0,
                           "trace_launches_per_step": int(st5.trace_launches) if st5 is not None else 0},
            }
            blk.update(multi_rank_fields(rep5, image_checksum(L5["full"], range(sd5.height), sd5.width),
                                         max(args.c5_steps, 1), distinct))
            device_error = device_error or blk["device_error"]
            out["c5"] = blk
        if emulated is not None:
            out["emulated_split"] = emulated
        if not args.no_cpu_baseline and world == 1:
            log("cpu baseline (oracle) ...")
            out["cpu_baseline"] = cpu_baseline(sd, cpu_threads(), args.cpu_rows, args.cpu_frames)
        if not args.no_golden:
            out["golden"] = golden_check()
            log(f"golden: {out['golden']['harness_pass']}/{out['golden']['scenes']} pass the reference harness, "
                f"max |delta| {out['golden']['max_abs_delta_non_glass']} (non-glass)")
        if args.verify:
            # rehearsal check: the gathered image equals one renderer drawing every row (bitwise)
            ref_r = scenes.make_renderer(sd)
            ref_r.set_params(**knobs)
            ref_r.draw_frames(sd.frames, TIME0, DTIME)
            ref_img = torch.from_numpy(ref_r.read_image())
            same = torch.equal(full.cpu().view(torch.int32), ref_img.view(torch.int32))
            out["verify_gather_bitwise"] = bool(same)
            log(f"verify: gathered image {'==' if same else '!='} single-renderer image")
        print(json.dumps(out), flush=True)
        if device_error:
            log(f"DEVICE CHECK FAILED: {device_error}")
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 3 if (rank == 0 and device_error) else 0


if __name__ == "__main__":
    sys.exit(main())
