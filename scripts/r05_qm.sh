#!/usr/bin/env bash
# Round-5 batch QM: the GPU suite with the dry-queue mask (a wave whose XCD's job queue ran dry skips the queues another
# wave already found dry), then same-box A/Bs against lib/libhrt_qm0.so (HRT_QMASK=0) on C2 (8-way split), C3, C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag="${1:-r05qm}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
export LIBS="lib/libhrt_qm0.so lib/libhrt.so"
{ bash scripts/ab_lib.sh "--steps 5" c2 && bash scripts/ab_lib.sh "--steps 3" c3 c4; } > "gpurun_out/$tag/ab_qmask.txt" 2>&1 || exit 1
cat "gpurun_out/$tag/ab_qmask.txt"
