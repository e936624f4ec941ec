#!/usr/bin/env bash
# Round-5 batch V: the cost order's head size (the share of tiles sorted most expensive first): 12 / 25 (product) / 50 /
# 100 % on the 8-way emulated splits of C4 and C2 (full images do not use the order), same box, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05v}"
mkdir -p "gpurun_out/$tag"
export LIBS="lib/libhrt_h12.so lib/libhrt.so lib/libhrt_h50.so lib/libhrt_h100.so"
bash scripts/ab_lib.sh "--steps 3" c4 c2 c3 > "gpurun_out/$tag/ab_head.txt" 2>&1 || exit 1
cat "gpurun_out/$tag/ab_head.txt"
