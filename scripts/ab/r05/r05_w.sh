#!/usr/bin/env bash
# Round-5 batch W (diagnostic build): C2's wave records with each wave's longest job but the last — is the last job of
# a 1/8 share's waves (~0.5 ms) long because of where it falls, or do jobs that long occur throughout the launch?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05w
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh r05w/wave_tail_c2 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 4 --full \
  --- r05w/wave_tail_c2_co1 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 4 --param cost_order=1 \
  --- r05w/wave_tail_c2_jf16 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 4 --param job_frames=16
