#!/usr/bin/env bash
# Round-6 batch V: the folding waves of fold 3 spread over the 8 XCDs (lib/libhrt.so) against all on one XCD
# (lib/libhrt_fold1xcd.so, -DHRT_FOLD_ONE_XCD: every 64th wave of the grid), C3 and C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06v}"
mkdir -p "gpurun_out/$tag"
LIBS="lib/libhrt_fold1xcd.so lib/libhrt.so" bash scripts/ab_lib.sh "--steps 5 --emulate-ranks 0" c3 2>&1 | tee "gpurun_out/$tag/ab_c3.txt"
LIBS="lib/libhrt_fold1xcd.so lib/libhrt.so" bash scripts/ab_lib.sh "--steps 1 --warmup 1 --emulate-ranks 0" c5 2>&1 | tee "gpurun_out/$tag/ab_c5.txt"
