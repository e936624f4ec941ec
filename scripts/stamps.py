"""Region time split of the render kernel from the diagnostic build's s_memtime stamps.

Run on the GPU box after `make -C hello-raytracing_amd diag`:
    HRT_LIB=lib/libhrt_diag.so python scripts/stamps.py --config c3 --frames 32 --variants 4 8

Prints, per variant, the share of summed wave cycles spent in closest-hit queries (traversal +
exact tests), shading (scatter + attenuation) and sample generation / accumulation, plus the
remainder: lane-cycles idle behind the wave's slowest lane (all sums are over lanes). The numbers are wave-cycle sums over all waves, so they are shares of the
issue time of the kernel, not of wall time; the diagnostic build itself perturbs scheduling a bit.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hello-raytracing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import hrt  # noqa: E402
from scenes import CONFIGS, make_renderer  # noqa: E402


def trace_summary(tr):
    """Residency timeline of one launch from the per-wave records (100 MHz ticks)."""
    import numpy as np
    st, en = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    ok = en > 0
    st, en = st[ok], en[ok]
    t0, t1 = st.min(), en.max()
    span = (t1 - t0) / 1e5  # ms
    life = (en - st) / 1e5
    edges = np.linspace(t0, t1, 41)
    conc = []
    for k in range(40):
        a, b = edges[k], edges[k + 1]
        ov = np.clip(np.minimum(en, b) - np.maximum(st, a), 0, None).sum() / (b - a)
        conc.append(round(float(ov) / 1024.0, 2))
    xcc = (tr[ok, 2] >> 32) & 0xF
    per_xcc = [round(float(life[xcc == k].sum()), 1) for k in range(8)]
    return {"span_ms": span, "life_ms_mean": float(life.mean()), "life_ms_p50": float(np.median(life)),
            "life_ms_p99": float(np.percentile(life, 99)), "life_ms_max": float(life.max()),
            "start_ms_last": float((st.max() - t0) / 1e5),
            "waves_per_simd_timeline": conc, "wave_ms_per_xcc": per_xcc}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--variants", type=int, nargs="+", default=[4])
    ap.add_argument("--fpl", type=int, nargs="+", default=[32], help="frames per launch (tiles schedule)")
    ap.add_argument("--schedule", type=int, default=2, help="1 tiles (k_render), 2 sample queue (k_trace)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--trace", default=None, help="directory for per-wave records (.npy)")
    a = ap.parse_args()
    L = hrt._lib.lib()
    if L.rt_diagnostic_build() != 1:
        raise SystemExit("not the diagnostic build: set HRT_LIB=lib/libhrt_diag.so")
    sd = CONFIGS[a.config]()
    rows = []
    for v, fpl in [(v, f) for v in a.variants for f in a.fpl]:
        r = make_renderer(sd)
        r.set_params(variant=v, frames_per_launch=fpl, schedule=a.schedule)
        r.draw_frames(2, 1000, 10)  # warm-up
        r.synchronize()
        r.draw_frames(a.frames, 1000, 10)
        r.synchronize()
        st = r.stats()
        q = r.raw_counters()
        trav, shade, gen, life = q[8], q[9], q[10], q[11]
        row = {
            "config": a.config, "variant": int(st.variant), "frames": a.frames, "fpl": fpl, "kernel_ms": st.kernel_ms,
            "rays": int(st.queries), "wave_cycles": int(life),
            "share_query": trav / life, "share_shade": shade / life, "share_gen": gen / life,
            "share_idle": 1.0 - (trav + shade + gen) / life,
            "lane_cycles_per_query": trav / max(1, st.queries),
            "primary_queries": int(q[5]), "box_tests_per_primary": q[6] / max(1, q[5]),
            "box_tests_per_secondary": (st.box_tests - q[6]) / max(1, st.queries - q[5]),
            "lane_cycles_per_primary": q[7] / max(1, q[5]),
            "lane_cycles_per_secondary": (trav - q[7]) / max(1, st.queries - q[5]),
            # s_memtime ticks per s_memrealtime tick (x 100 MHz = memtime clock), and the mean number of
            # resident waves per SIMD over the draw (wave-lifetime sum / (draw time x 1024 SIMDs))
            "memtime_mhz": 100.0 * q[14] / max(1, q[12]),
            "waves": int(q[13]),
            "resident_waves_per_simd": (q[12] / 1e8) / (st.trace_ms / 1e3) / 1024.0,
        }
        if a.trace and a.schedule == 1:
            import numpy as np
            nw = 8 * ((sd.width + 15) // 16) * ((sd.height + 15) // 16) * 4
            buf = (hrt._lib.C.c_uint64 * nw)()
            hrt._lib.check(L.rt_get_wave_trace(r._h, buf, nw), "wave_trace")
            tr = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:, :4].copy()
            name = os.path.join(a.trace, f"trace_{a.config}_v{v}_f{fpl}.npy")
            np.save(name, tr)
            row.update(trace_summary(tr))
        rows.append(row)
        print(json.dumps(row), flush=True)
        r.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"time": time.time(), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
