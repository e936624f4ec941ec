"""Generate tests/golden/oracle/: float32 outputs of the CPU oracle (oracle/rt_oracle.c) for row subsets of
every BASELINE config and of the golden / triangle scenes (SURVEY §8(c) "golden vectors to commit"), and
digests of the host tree builds. Run in the build container after changing nothing in the oracle:

    python tests/golden/make_oracle_fixtures.py

The oracle itself is pinned to the reference's golden images (tests/test_oracle_golden.py); these files pin
it in time (tests/test_oracle_fixtures.py re-renders them bit for bit) and give the GPU tests a stored
expected output (tests/test_gpu_parity.py::test_hip_reproduces_oracle_fixtures). Data only: images,
ray counts, triangle-program work counts and SHA-256 digests.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
for p in (ROOT, ROOT / "hello-raytracing_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))

import scenes  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main() -> int:
    out = scenes.ORACLE_FIXTURE_DIR
    out.mkdir(parents=True, exist_ok=True)
    images, manifest = {}, {}
    for name, (sd, (row0, step)) in scenes.oracle_fixture_cases().items():
        nrows = len(range(row0, sd.height, step))
        img, q = scenes.oracle_render(sd, rows=(row0, step, nrows))
        images[name] = img
        manifest[name] = {"width": sd.width, "height": sd.height, "mode": sd.mode, "frames": sd.frames,
                          "row0": row0, "row_step": step, "nrows": nrows, "queries": q,
                          "node_tests": int(O.last_counts["node_tests"]), "tri_tests": int(O.last_counts["tri_tests"]),
                          "capped_walks": int(O.last_counts["capped_walks"])}
        print(name, img.shape, q, O.last_counts, flush=True)
    np.savez_compressed(out / "images.npz", **images)
    (out / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=True) + "\n")
    trees = {name: scenes.tree_digest(build()) for name, build in scenes.oracle_fixture_trees().items()}
    (out / "trees.json").write_text(json.dumps(trees, indent=1, sort_keys=True) + "\n")
    print("trees", {k: v["sizes"] for k, v in trees.items()})
    return 0


if __name__ == "__main__":
    sys.exit(main())
