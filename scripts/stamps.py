"""Region time split of the render kernel from the diagnostic build's s_memtime stamps.

Run on the GPU box after `make -C hello-raytracing_amd diag`:
    HRT_LIB=lib/libhrt_diag.so python scripts/stamps.py --config c3 --frames 32 --variants 4 8

Prints, per variant, the share of summed wave cycles spent in closest-hit queries (traversal +
exact tests), shading (scatter + attenuation) and sample generation / accumulation, plus the
loop-external remainder. The numbers are wave-cycle sums over all waves, so they are shares of the
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--variants", type=int, nargs="+", default=[4])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    L = hrt._lib.lib()
    if L.rt_diagnostic_build() != 1:
        raise SystemExit("not the diagnostic build: set HRT_LIB=lib/libhrt_diag.so")
    sd = CONFIGS[a.config]()
    rows = []
    for v in a.variants:
        r = make_renderer(sd)
        r.set_params(variant=v)
        r.draw_frames(2, 1000, 10)  # warm-up
        r.synchronize()
        r.draw_frames(a.frames, 1000, 10)
        r.synchronize()
        st = r.stats()
        q = r.raw_counters()
        trav, shade, gen, life = q[8], q[9], q[10], q[11]
        row = {
            "config": a.config, "variant": int(st.variant), "frames": a.frames, "kernel_ms": st.kernel_ms,
            "rays": int(st.queries), "wave_cycles": int(life),
            "share_query": trav / life, "share_shade": shade / life, "share_gen": gen / life,
            "share_other": 1.0 - (trav + shade + gen) / life,
            "cycles_per_query_wave": trav / max(1, st.queries) * 64,
        }
        rows.append(row)
        print(json.dumps(row), flush=True)
        r.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"time": time.time(), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
