"""Lane utilisation of k_trace_split's walk and shading phases (diagnostic build counters 5-14).

Run on the GPU box after `make -C hello-raytracing_amd diag`:
    HRT_LIB=lib/libhrt_diag.so python scripts/diag_split.py [--suspend 0 8 16 32]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "hello-raytracing_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))
import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--suspend", type=int, nargs="+", default=[1, 8, 16, 24, 32, 48])
ap.add_argument("--frames", type=int, default=64)
a = ap.parse_args()
sd = scenes.config_c3(1920, 1080, a.frames)
for sb in a.suspend:
    r = scenes.make_renderer(sd)
    r.set_params(variant=4, schedule=2, suspend_below=sb)
    r.draw_frames(sd.frames, 1000, 10)
    st = r.stats()
    c = r.raw_counters()
    lbox, wbox, lleaf, wleaf, rounds, lshade, wshade, lwalk, wwalk, lentry = c[5:15]
    print(f"suspend_below {sb:2d}: {st.trace_ms:8.1f} ms  box-step util {lbox / max(64 * wbox, 1):.3f}  "
          f"leaf-step util {lleaf / max(64 * wleaf, 1):.3f}  box steps/query {lbox / st.queries:.2f} "
          f"wave box steps/query {64 * wbox / st.queries:.2f}  leaf {lleaf / st.queries:.2f}/{64 * wleaf / st.queries:.2f}  "
          f"rounds/query/64 {64 * rounds / st.queries:.3f}  shading lanes/round {lshade / max(wshade, 1):.1f}  "
          f"walking lanes per walk iteration {lwalk / max(wwalk, 1):.1f}  lanes entering the walk per round "
          f"{lentry / max(rounds, 1):.1f}", flush=True)
