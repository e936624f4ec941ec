#!/usr/bin/env bash
# Round-5 phase splits of the split kernels (diagnostic phase build) for C3 / C4 / C5 at 16 frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r05_phase
HRT_LIB=lib/libhrt_phase.so bash scripts/gpu_step.sh r05_phase/c3 300 python scripts/phase_split.py --config c3 --frames 16 \
  --- r05_phase/c4 300 python scripts/phase_split.py --config c4 --frames 16 \
  --- r05_phase/c5 300 python scripts/phase_split.py --config c5 --frames 16
