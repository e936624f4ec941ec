#!/usr/bin/env bash
# Round-5 final check B: the GPU parity suite on the final tree, then the round's profiles (scripts/profile_r05.sh:
# rocprofv3 kernel-trace stats + PMC passes of C3 / C4 / C5 and the phase splits).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05_final3}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
bash scripts/ab/r05/profile_r05.sh
