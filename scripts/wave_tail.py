"""Where a short launch loses its time: per-wave records of the suspendable-walk kernels (diagnostic build).

Run on the GPU box after `make -C hello-raytracing_amd diag`:
    HRT_LIB=lib/libhrt_diag.so python scripts/wave_tail.py --config c4 --ranks 8 --rank 4

Draws one rank's share of the N-way row split (bench.py's partition) and the full image with the bench's timed knobs,
and summarises each draw's LAST trace launch from its wave records (rt_get_wave_trace): launch span, when waves
started and when they first found no frame block left (the queue drain), their end times, the resident waves over
time, and frame blocks per wave. Tells a launch's fixed costs (ramp, drain tail) from a slower per-ray rate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "hello-raytracing_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import bench  # noqa: E402
import hrt  # noqa: E402
import scenes  # noqa: E402
from hrt.parallel import owned_rows, rank_params  # noqa: E402


def summarise(tr: np.ndarray) -> dict:
    st, en = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    ok = en > 0
    st, en, info = st[ok], en[ok], tr[ok, 3].astype(np.int64)
    drained = info & 0xFFFFFFFF
    blocks = info >> 32  # frame blocks generated (split kernels) or jobs taken (k_trace)
    clk0, clk1, w6, w7 = (tr[ok, k].astype(np.int64) for k in (4, 5, 6, 7))
    dclk, jclk = w6 & 0xFFFFFFFF, w6 >> 32  # shader-clock ticks from start to the drain / to the last job take
    last_job = (tr[ok, 2].astype(np.uint64) >> np.uint64(40)).astype(np.int64)  # k_trace: when the last job was taken
    xcc = (tr[ok, 2] >> 32) & 0xFF
    t0 = st.min()
    span = (en.max() - t0) / 1e5
    pct = lambda a: [round(float(np.percentile(a, q)), 3) for q in (0, 10, 50, 90, 100)]  # noqa: E731
    edges = np.linspace(t0, en.max(), 26)
    conc = []
    for k in range(25):
        a, b = edges[k], edges[k + 1]
        conc.append(round(float(np.clip(np.minimum(en, b) - np.maximum(st, a), 0, None).sum() / (b - a)), 1))
    return {
        "waves": int(ok.sum()),
        "span_ms": round(float(span), 3),
        "start_ms_pcts": pct((st - t0) / 1e5),
        "drain_ms_pcts": pct((st + drained - t0) / 1e5),
        "end_ms_pcts": pct((en - t0) / 1e5),
        "tail_after_first_drain_ms": round(float((en.max() - (st + drained).min()) / 1e5), 3),
        ("jobs_per_wave_pcts" if last_job.any() else "blocks_per_wave_pcts"): pct(blocks),
        "last_job_ms_pcts": pct((st + last_job - t0) / 1e5) if last_job.any() else None,
        "last_job_to_end_ms_pcts": pct((en - st - last_job) / 1e5) if last_job.any() else None,
        # k_trace: the longest time between two of the wave's job fetches (its longest job but the last)
        "max_job_ms_pcts": pct((tr[ok, 2].astype(np.int64) & 0xFFFFFF) / 1e5) if last_job.any() else None,
        ("jobs_total" if last_job.any() else "blocks_total"): int(blocks.sum()),
        # shader clock (s_memtime ticks per s_memrealtime tick x 100 MHz) over each wave's life and after its drain
        "clock_mhz_pcts": pct((clk1 - clk0) / np.maximum(en - st, 1) * 100.0),
        "clock_mhz_after_drain_pcts": pct((clk1 - clk0 - dclk)[dclk > 0] / np.maximum((en - st - drained)[dclk > 0], 1) * 100.0)
        if (dclk > 0).any() else None,
        # k_trace: lanes holding a sample when the wave found the queue drained, samples finished after its last job take,
        # rounds after the drain, rounds from the last job take to the drain, shader cycles per round then and overall
        "inflight_at_drain_pcts": pct(w7 & 0xFF) if last_job.any() else None,
        "finished_after_last_job_pcts": pct((w7 >> 8) & 0xFFFF) if last_job.any() else None,
        "rounds_after_drain_pcts": pct((w7 >> 24) & 0xFFF) if last_job.any() else None,
        "rounds_in_last_job_pcts": pct((w7 >> 36) & 0xFFF) if last_job.any() else None,
        "clk_per_round_last_job_pcts": pct((dclk - jclk)[dclk > 0] / np.maximum((w7 >> 36) & 0xFFF, 1)[dclk > 0])
        if last_job.any() and (dclk > 0).any() else None,
        "clk_per_round_overall_pcts": pct((clk1 - clk0) / np.maximum(w7 >> 48, 1)) if last_job.any() else None,
        "resident_waves_timeline": conc,
        # by dispatch order (wave index deciles: the first-dispatched waves are the oldest on their SIMD), p50 of the last
        # job's length (k_trace), of the jobs taken and of the end time
        "by_dispatch_decile": [{"last_job_to_end_ms_p50": round(float(np.median((en - st - last_job)[g] / 1e5)), 3)
                                if last_job.any() else None,
                                "jobs_p50": float(np.median(blocks[g])), "end_ms_p50": round(float(np.median((en - t0)[g] / 1e5)), 3)}
                               for g in np.array_split(np.arange(len(st)), 10)],
        # per XCD (XCC_ID): end time and the last job's length (k_trace), p50 / p100
        "by_xcd": {int(x): {"end_ms": [round(float(np.percentile((en - t0)[xcc == x] / 1e5, q)), 3) for q in (50, 100)],
                            "last_job_to_end_ms": [round(float(np.percentile((en - st - last_job)[xcc == x] / 1e5, q)), 3)
                                                   for q in (50, 100)] if last_job.any() else None,
                            "waves": int((xcc == x).sum())}
                   for x in np.unique(xcc)},
    }


def draw(sd, params: dict):
    r = scenes.make_renderer(sd)
    r.set_params(**params)
    for _ in range(2):  # warm, then the recorded draw
        r.reset_frame_count()
        r.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
        r.synchronize()
    t = time.perf_counter()
    r.reset_frame_count()
    r.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
    st = r.stats()
    wall = time.perf_counter() - t
    import ctypes as C
    words = 8 * 32 * 256
    buf = (C.c_uint64 * words)()
    hrt._lib.check(hrt.lib().rt_get_wave_trace(r._h, buf, words), "rt_get_wave_trace")
    tr = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
    out = {"kernel": st.kernel.decode(), "trace_ms": round(st.trace_ms, 3), "kernel_ms": round(st.kernel_ms, 3),
           "wall_ms": round(wall * 1e3, 3), "trace_launches": st.trace_launches, "rays": st.queries}
    out.update(summarise(tr))
    if out.get("jobs_total"):  # k_trace: per-job records after the wave records (renderer.cpp, job_trace)
        p = r.params
        nrows = len(owned_rows(p.row0, p.row_step, sd.height, p.row_block))
        wave_words = 8 * max(((sd.width + 15) // 16) * ((nrows + 15) // 16) * 4, 32 * 256)
        tiles_w, tiles = (sd.width + 7) // 8, ((sd.width + 7) // 8) * ((nrows + 7) // 8)
        nj = out["jobs_total"]
        jb = (C.c_uint64 * (wave_words + nj))()
        hrt._lib.check(hrt.lib().rt_get_wave_trace(r._h, jb, wave_words + nj), "rt_get_wave_trace")
        jt = np.frombuffer(jb, dtype=np.uint64)[wave_words:].astype(np.int64)
        out["jobs"] = summarise_jobs(jt, tiles_w, tiles, nj // tiles, tr)
    return out


def summarise_jobs(jt: np.ndarray, tiles_w: int, tiles: int, nchunks: int, tr: np.ndarray) -> dict:
    """Each job's duration (take to the wave's next take or drain) against when it was taken and where its tile is."""
    ok = jt != 0
    dur = (jt & 0xFFFFFFFF)[ok] / 1e5  # ms
    t0 = tr[:, 0][tr[:, 1] > 0].min() & 0xFFFFFFFF
    at = (((jt >> 32) - t0) % (1 << 32))[ok] / 1e5
    job = np.nonzero(ok)[0]
    row = (job // max(nchunks, 1)) // tiles_w  # tile row
    pct = lambda a: [round(float(np.percentile(a, q)), 3) for q in (10, 50, 90, 99)] if len(a) else None  # noqa: E731
    edges = np.percentile(at, [0, 50, 80, 90, 95, 98, 100])
    by_time = {f"{edges[k]:.2f}-{edges[k + 1]:.2f} ms": pct(dur[(at >= edges[k]) & (at <= edges[k + 1])])
               for k in range(len(edges) - 1)}
    rows = np.unique(row)
    groups = np.array_split(rows, min(10, len(rows)))
    by_row = {f"tile rows {g[0]}-{g[-1]}": pct(dur[np.isin(row, g)]) for g in groups}
    late = at >= edges[-3]  # the last 5 % of takes
    late_rows = np.unique(row[late])
    same_rows_early = np.isin(row, late_rows) & ~late
    return {"recorded": int(ok.sum()), "duration_ms_pcts_by_take_time": by_time, "duration_ms_pcts_by_tile_row": by_row,
            "last_5pct_takes": {"tile_rows": [int(late_rows.min()), int(late_rows.max())] if late.any() else None,
                                "duration_ms_pcts": pct(dur[late]),
                                "same_rows_taken_earlier_ms_pcts": pct(dur[same_rows_early])}}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--rank", type=int, nargs="+", default=[4])
    ap.add_argument("--steal", type=int, default=None)
    ap.add_argument("--full", action="store_true", help="also the full image")
    ap.add_argument("--param", action="append", default=[], help="extra rt_params field=value (repeatable)")
    a = ap.parse_args()
    assert hrt.lib().rt_diagnostic_build() == 1, "run with HRT_LIB=lib/libhrt_diag.so"
    sd = scenes.CONFIGS[a.config]()
    extra = {} if a.steal is None else {"steal": a.steal}
    extra.update({k: int(v) for k, v in (p.split("=", 1) for p in a.param)})
    res = {}
    for k in a.rank:
        res[f"rank{k}of{a.ranks}"] = draw(sd, {**rank_params(k, a.ranks, 8), **bench.timed_knobs(**extra)})
    if a.full:
        res["full"] = draw(sd, {**rank_params(0, 1, 8), **bench.timed_knobs(**extra)})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
