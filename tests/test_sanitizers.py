"""Sanitizer build of the host-side code and the CPU oracle.

tests/native/host_check.cpp links the host builders (OBJ ingest, Tree::build, the sphere / triangle BVH builders,
render_ppm / compare_ppm_images: hello-raytracing_amd/csrc/host) and oracle/rt_oracle.c compiled with
-fsanitize=address,undefined (every UBSan finding fatal) and drives them over every shipped asset, a corpus of
malformed OBJ inputs (truncated faces, index 0, huge / negative / wrapping indices, non-UTF-8 bytes, hex and
nan(...) floats) and 3000 seeded random mutations of the assets. A standalone executable rather than the
Python suite under an LD_PRELOADed runtime: the sanitizer runtime is linked into the driver itself. Found on
the first run: a null-pointer member access in Tree::build on an empty mesh, and (by the corpus) a size_t wrap
in the face-index bound check of the OBJ parser that let a crafted index read out of bounds.
"""
import gzip
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
NATIVE = ROOT / "tests" / "native"


def test_host_code_and_oracle_clean_under_asan_ubsan(tmp_path):
    subprocess.run(["make", "-s", "-C", str(NATIVE), "SAN=1"], check=True, timeout=600)
    for f in (ROOT / "hello-raytracing_amd" / "assets").glob("*.obj.gz"):
        (tmp_path / f.name[:-3]).write_bytes(gzip.decompress(f.read_bytes()))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([str(NATIVE / "build" / "san" / "host_check"), str(tmp_path), "3000"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-6000:])
    assert "host_check: 0 failures" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-6000:]
    assert "suzanne.obj: 515 vertices, 2937 indices" in p.stdout  # mesh.rs:80-88 pin, under the sanitizers
