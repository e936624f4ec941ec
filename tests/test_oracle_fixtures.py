"""The committed oracle fixtures (tests/golden/oracle, SURVEY §8(c) golden vectors) against the oracle and
the host builders as they are now: every image bit, ray count and triangle-program work count, and the
SHA-256 of every tree build. CPU only. The GPU side of the same fixtures is
tests/test_gpu_parity.py::test_hip_reproduces_oracle_fixtures."""
import json

import numpy as np
import pytest

import scenes
from oracle import oracle as O

CASES = scenes.oracle_fixture_cases()


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_reproduces_fixture(name):
    sd, (row0, step) = CASES[name]
    want, man = scenes.load_oracle_fixture(name)
    img, q = scenes.oracle_render(sd, rows=(row0, step, man["nrows"]))
    assert (sd.width, sd.height, sd.frames, sd.mode) == (man["width"], man["height"], man["frames"], man["mode"])
    np.testing.assert_array_equal(img.view(np.uint32), want.view(np.uint32))
    assert q == man["queries"]
    assert (O.last_counts["node_tests"], O.last_counts["tri_tests"], O.last_counts["capped_walks"]) == \
        (man["node_tests"], man["tri_tests"], man["capped_walks"])


def test_tree_builds_match_fixture_digests():
    want = json.loads((scenes.ORACLE_FIXTURE_DIR / "trees.json").read_text())
    trees = scenes.oracle_fixture_trees()
    assert sorted(want) == sorted(trees)
    for name, build in trees.items():
        assert scenes.tree_digest(build()) == want[name], name
    # the reference's own structural pins (src/scene/bvh/tree.rs:107-110, :121-124)
    assert want["cube"]["sizes"] == [16, 12] and want["suzanne"]["sizes"] == [1024, 979]


def test_fixture_set_covers_every_config_and_the_step_cap():
    man = json.loads((scenes.ORACLE_FIXTURE_DIR / "manifest.json").read_text())
    assert {"c1", "c2", "c3", "c4", "c5"} <= set(man)
    assert man["tris_dragon"]["capped_walks"] > 0  # the 600-step cap binds inside the fixture
