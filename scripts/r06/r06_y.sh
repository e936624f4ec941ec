#!/usr/bin/env bash
# Round-6 batch Y: fold 3's folding share with the XCD-spread placement: 1 in 32 / 64 (product) / 128 waves, C3, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06y}"
mkdir -p "gpurun_out/$tag"
LIBS="lib/libhrt_fm32.so lib/libhrt.so lib/libhrt_fm128.so" bash scripts/ab_lib.sh "--steps 5 --emulate-ranks 0" c3 2>&1 | tee "gpurun_out/$tag/ab_c3.txt"
