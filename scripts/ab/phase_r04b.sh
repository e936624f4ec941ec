#!/usr/bin/env bash
# Phase split of the final round-4 tree (diagnostic build lib/libhrt_phase.so, -DHRT_STAMPS -DHRT_PHASES): C3 at
# 1024 frames, C4 at 512, C5 at 16.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/phase_r04b
mkdir -p $o
HRT_LIB=lib/libhrt_phase.so timeout -k 10 300 python scripts/phase_split.py --config c3 --frames 1024 > $o/c3_1024f.log 2>&1 &&
HRT_LIB=lib/libhrt_phase.so timeout -k 10 300 python scripts/phase_split.py --config c4 --frames 512 > $o/c4_512f.log 2>&1 &&
HRT_LIB=lib/libhrt_phase.so timeout -k 10 300 python scripts/phase_split.py --config c5 --frames 16 > $o/c5_16f.log 2>&1
for f in $o/*.log; do tail -1 "$f"; done
