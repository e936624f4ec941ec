#!/usr/bin/env bash
# Round-5 batch Q: the GPU suite with per-XCD job queues (sample buffer), then same-box A/Bs against
# lib/libhrt_nq0.so (HRT_NQ=0: one job counter for the GPU): C2 (16- and 8-frame jobs), C3, C4 and C5 (256 spp),
# with the 8-way emulated splits where they run by default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05q}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
export LIBS="lib/libhrt_nq0.so lib/libhrt.so"
{ bash scripts/ab_lib.sh "--steps 5" c2 && bash scripts/ab_lib.sh "--steps 5 --job-frames 8" c2 \
  && bash scripts/ab_lib.sh "--steps 3" c3 c4 && bash scripts/ab_lib.sh "--steps 2 --frames 256 --emulate-ranks 0" c5; } \
  > "gpurun_out/$tag/ab_nq.txt" 2>&1 || exit 1
cat "gpurun_out/$tag/ab_nq.txt"
