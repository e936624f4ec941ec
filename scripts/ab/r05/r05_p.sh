#!/usr/bin/env bash
# Round-5 batch P: the GPU suite, then same-box A/Bs of the owner's claim size for jobs dealt early (STEAL_OWN_EARLY 4,
# the product, against lib/libhrt_oe1.so = 1 frame per claim as before): C4 with its 8-way emulated split (stealing
# auto), and full images with stealing forced on (--steal 2: the claims' cost) for C4 and C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05p}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
export LIBS="lib/libhrt_oe1.so lib/libhrt.so"
{ bash scripts/ab_lib.sh "--steps 3" c4 && bash scripts/ab_lib.sh "--steps 3 --steal 2 --emulate-ranks 0" c4 c3; } \
  > "gpurun_out/$tag/ab_own_early.txt" 2>&1 || exit 1
cat "gpurun_out/$tag/ab_own_early.txt"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c4" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0
