#!/usr/bin/env bash
# Round-5 batch H (diagnostic build): wave records of C2's 1/8 shares and full image (k_trace), and the lanes of the
# mixed kernel's begin-phase sphere walk on C5 (scripts/diag_tris.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05h}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c2" 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 4 0 --full \
  --- "$tag/diag_tris_c5" 300 python scripts/diag_tris.py --frames 16
