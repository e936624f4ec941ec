#!/usr/bin/env bash
# Round-6 batch PH: phase split (diagnostic build lib/libhrt_phase.so) of C3 with the two-pass leaf, C4 and C5, 16 frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06ph}"
mkdir -p "gpurun_out/$tag"
for c in c3 c4 c5; do
  HRT_LIB=lib/libhrt_phase.so timeout -k 10 300 python scripts/phase_split.py --config $c --frames 16 > "gpurun_out/$tag/phase_$c.log" 2>&1 || exit 1
  tail -1 "gpurun_out/$tag/phase_$c.log"
done
