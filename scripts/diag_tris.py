"""The mixed kernel's begin-phase sphere walk (k_trace_split_tris, run to completion; diagnostic build counters 5-14).

Run on the GPU box after `make -C hello-raytracing_amd diag`:
    HRT_LIB=lib/libhrt_diag.so python scripts/diag_tris.py [--frames 16]

For C5's scene (4K, the bench's knobs) prints the sphere walk's lanes per box / leaf step, the lanes that enter it per
walk, and the share of its wave steps run with fewer than 24 lanes (DIAG_LOW in bvh_run) — the part of the walk a
suspendable sphere walk (threshold 24, as the heap walk's) would move into fuller steps.
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "hello-raytracing_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))
import bench  # noqa: E402
import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=16)
a = ap.parse_args()
sd = scenes.config_c5(frames=a.frames)
r = scenes.make_renderer(sd)
r.set_params(**bench.timed_knobs())
r.draw_frames(sd.frames, bench.TIME0, bench.DTIME)
st = r.stats()
c = r.raw_counters()
lbox, wbox, lleaf, wleaf, lbox_low, wbox_low, lleaf_low, wleaf_low, lentry, wentry = c[5:15]
q = max(st.queries, 1)
print(f"kernel {st.kernel.decode()}  trace {st.trace_ms:.1f} ms  queries {st.queries}")
print(f"begin walks (waves) {wentry}  lanes entering per walk {lentry / max(wentry, 1):.1f}")
print(f"box steps: lanes per wave step {lbox / max(wbox, 1):.1f}  wave steps/query {64 * wbox / q:.2f}  "
      f"lane steps/query {lbox / q:.2f}  wave steps with < 24 lanes {wbox_low / max(wbox, 1):.3f} "
      f"(lanes in them per step {lbox_low / max(wbox_low, 1):.1f})")
print(f"leaf steps: lanes per wave step {lleaf / max(wleaf, 1):.1f}  wave steps/query {64 * wleaf / q:.2f}  "
      f"wave steps with < 24 lanes {wleaf_low / max(wleaf, 1):.3f} (lanes {lleaf_low / max(wleaf_low, 1):.1f})")
