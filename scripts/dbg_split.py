"""Work counters of k_trace vs k_trace_split on a small C3 render (debug aid)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "hello-raytracing_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))
import numpy as np
import scenes

sd = scenes.config_c3(190, 106, 5)
base = None
for sb in (0, 1, 8, 32, 64):
    r = scenes.make_renderer(sd)
    r.set_params(variant=4, schedule=2, suspend_below=sb)
    r.draw_frames(sd.frames, 1000, 10)
    st = r.stats()
    img = r.read_image()
    same = base is None or np.array_equal(img.view(np.uint32), base.view(np.uint32))
    if base is None:
        base = img
    print(f"sb={sb}: queries {st.queries} boxes {st.box_tests} spheres {st.sphere_tests} same={same}", flush=True)
    print("   raw", r.raw_counters()[:8] if hasattr(r, "raw_counters") else None, flush=True)
