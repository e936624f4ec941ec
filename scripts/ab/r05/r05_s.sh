#!/usr/bin/env bash
# Round-5 batch S (diagnostic build): wave records of C4's 1/8 shares 4 and 0 with 16-frame jobs (stealing off by the auto
# rule, cost order on by the auto rule), the same in raster order, and the default (32-frame jobs, stealing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05s}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/c4_jf16" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 5 --param job_frames=16 \
  --- "$tag/c4_jf16_raster" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 5 --param job_frames=16 --param cost_order=1 \
  --- "$tag/c4_default" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 5
