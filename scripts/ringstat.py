"""Fold-ring statistics of the diagnostic build (make EXTRA=-DHRT_RINGSTAT -> lib/libhrt_ringstat.so).

usage: HRT_LIB=lib/libhrt_ringstat.so python scripts/ringstat.py c3 [c2 c4 ...] [--budget MB] [--jf N]
Prints per config: draw time, waves' rounds stalled on an older job, rounds waiting for a ring slot, folds and
the mean fold time (cycles).
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "hello-raytracing_amd"), str(ROOT / "tests")]
import hrt  # noqa: E402
import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("configs", nargs="+")
ap.add_argument("--budget", type=int, default=512)
ap.add_argument("--jf", type=int, default=None)
a = ap.parse_args()
for cfg in a.configs:
    sd = scenes.CONFIGS[cfg]()
    r = scenes.make_renderer(sd)
    kw = {"schedule": hrt.RT_SCHEDULE_QUEUE}
    if a.budget:
        kw["queue_budget_mb"] = a.budget
    if a.jf:
        kw["job_frames"] = a.jf
    r.set_params(**kw)
    r.draw_frames(sd.frames, 1000, 10)
    st = r.stats()
    c = r.raw_counters(16)
    folds = max(c[7], 1)
    print(f"{cfg}: {st.kernel_ms:.1f} ms kernel {st.kernel.decode()} fold {'ring' if st.fold_ring else 'buffer'} {st.fold_bytes / 2**20:.0f} MiB "
          f"launches {st.launches}: stall rounds {c[5]}, slot-wait rounds {c[6]}, folds {c[7]}, "
          f"fold {16 * c[8] / folds:.0f} cycles each ({16 * c[8] / 1e9:.2f} G wave-cycles)", flush=True)
