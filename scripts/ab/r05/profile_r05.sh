#!/usr/bin/env bash
# Round-5 profiles of C3 / C4 / C5 on the final tree: rocprofv3 kernel-trace stats + the PMC passes (scripts/profile_round.sh)
# and the phase split of the diagnostic phase build (C3, C4, C5 at 16 frames; lib/libhrt_phase.so). Logs: gpurun_out/r05_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash scripts/profile_round.sh r05_c3 --config c3 --steps 3 --warmup 1 --emulate-ranks 0 &&
bash scripts/profile_round.sh r05_c4 --config c4 --steps 3 --warmup 1 --emulate-ranks 0 &&
bash scripts/profile_round.sh r05_c5 --config c5 --steps 1 --warmup 1 --emulate-ranks 0 &&
mkdir -p gpurun_out/r05_phase &&
HRT_LIB=lib/libhrt_phase.so bash scripts/gpu_step.sh r05_phase/c3 300 python scripts/phase_split.py --config c3 --frames 16 \
  --- r05_phase/c4 300 python scripts/phase_split.py --config c4 --frames 16 \
  --- r05_phase/c5 300 python scripts/phase_split.py --config c5 --frames 16
