#!/usr/bin/env bash
# Round-6 batch J: C2 with s_setprio(3) for waves holding one of the launch's last jobs (lib/libhrt_tailprio.so), same-box
# A/B against the product library (full image; the emulated split's shares deal in cost order, unaffected).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06j}"
mkdir -p "gpurun_out/$tag"
LIBS="lib/libhrt.so lib/libhrt_tailprio.so" bash scripts/ab_lib.sh "--steps 10 --emulate-ranks 0" c2 2>&1 | tee "gpurun_out/$tag/ab.txt"
