"""Phase split of k_trace_split_tris (triangle / mixed programs) from the diagnostic build's stamps.

Build the phase library here (it travels with the tree):
    make -C hello-raytracing_amd BUILD=build_phase LIB=lib/libhrt_phase.so EXTRA="-DHRT_STAMPS -DHRT_PHASES" lib/libhrt_phase.so
and run on the GPU box:
    HRT_LIB=lib/libhrt_phase.so python scripts/phase_split.py --config c5 --frames 16

Prints the share of wave cycles per phase of the split kernels' round loop (k_trace_split, k_trace_split_tris) —
refill (frame-block primary rays, job bookkeeping), begin (bvh_begin; the mixed program's whole sphere scan +
heap_begin), walk (the suspendable culling-BVH or heap walk), shade (hit record, scatter, colour store, job
accounting) — and the lanes active in the begin and shade phases.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hello-raytracing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import hrt  # noqa: E402
from scenes import CONFIGS, make_renderer  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--suspend-below", type=int, nargs="+", default=[None])
    ap.add_argument("--packet", type=int, default=0, help="rt_params.packet (sphere program): 0 auto, 1 off, 2 on")
    a = ap.parse_args()
    if hrt._lib.lib().rt_diagnostic_build() != 1:
        raise SystemExit("not a diagnostic build: set HRT_LIB=lib/libhrt_phase.so")
    sd = CONFIGS[a.config]()
    for sb in a.suspend_below:
        r = make_renderer(sd)
        r.set_params(schedule=hrt.RT_SCHEDULE_QUEUE, fold=hrt.RT_FOLD_BUFFER, packet=a.packet,
                     **({} if sb is None else {"suspend_below": sb}))
        r.draw_frames(2, 1000, 10)  # warm-up
        r.synchronize()
        r.draw_frames(a.frames, 1000, 10)
        r.synchronize()
        st = r.stats()
        q = r.raw_counters()
        life = q[12]
        row = {"config": a.config, "frames": a.frames, "kernel": st.kernel.decode(), "suspend_below": st.suspend_below,
               "kernel_ms": round(st.kernel_ms, 3), "rays": int(st.queries),
               "share": {k: round(q[8 + i] / life, 4) for i, k in enumerate(["refill", "begin", "walk", "shade"])},
               "begin_lanes": round(q[5] / max(q[13], 1), 2), "shade_lanes": round(q[7] / max(q[14], 1), 2),
               "rays_per_wave_cycle_e6": round(st.queries / life * 1e6, 2),
               "node_tests_per_ray": round(st.node_tests / st.queries, 2),
               "tri_tests_per_ray": round(st.tri_tests / st.queries, 2),
               "sphere_tests_per_ray": round(st.sphere_tests / st.queries, 2),
               "box_tests_per_ray": round(st.box_tests / st.queries, 2)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
