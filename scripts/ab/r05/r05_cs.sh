#!/usr/bin/env bash
# Round-5 batch CS: the GPU parity suite with the work counters spread over 64 copies, then same-box A/Bs against
# lib/libhrt_cs1.so (HRT_CSPREAD=1: every wave adds to one set, as before) on C2 / C3 / C4 / C5 (256 spp), and C2's
# 8-way split, plus the wave records of C2's 1/8 shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag="${1:-r05cs}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
export LIBS="lib/libhrt_cs1.so lib/libhrt.so"
{ bash scripts/ab_lib.sh "--steps 5" c2 && bash scripts/ab_lib.sh "--steps 3 --emulate-ranks 0" c3 c4 \
  && bash scripts/ab_lib.sh "--steps 2 --frames 256 --emulate-ranks 0" c5; } > "gpurun_out/$tag/ab_cspread.txt" 2>&1 || exit 1
cat "gpurun_out/$tag/ab_cspread.txt"
