"""pytest configuration: import paths and the `gpu` marker.

`-m "not gpu"` runs on any host (oracle vs the reference's goldens, host-side builders, C-ABI load check);
`-m gpu` needs an MI355X and compares the HIP path with the oracle through the C-ABI.
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "hello-raytracing_amd", ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU oracle renders")
