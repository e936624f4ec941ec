#!/usr/bin/env bash
# Round-5 batch: the short-launch / walk-lane diagnostics (scripts/r05_tail.sh), then k_trace_split with 896-lane
# workgroups (nodes in LDS; + leaf spheres in LDS) against the product build: C3 parity tests on the variant, then an
# interleaved same-box A/B (scripts/ab_lib.sh). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05c}"
mkdir -p "gpurun_out/$tag"
bash scripts/r05_tail.sh "$tag" || exit 1
HRT_LIB=lib/libhrt_wg896.so bash scripts/gpu_step.sh "$tag/wg896_tests" 300 python -u -m pytest tests/test_gpu_timed.py \
  "tests/test_gpu_parity.py::test_full_size_headline_configs_agree" "tests/test_gpu_parity.py::test_hip_reproduces_oracle_fixtures" \
  "tests/test_gpu_parity.py::test_golden_scene_full_draw_sample_queue" "tests/test_gpu_parity.py::test_work_stealing_bit_identical" \
  -x -q --timeout 200 --timeout-method thread || exit 1
LIBS="lib/libhrt.so lib/libhrt_wg896.so lib/libhrt_wg896n.so" bash scripts/ab_lib.sh "--steps 5" c3 > "gpurun_out/$tag/ab_wg896.txt" 2>&1
cat "gpurun_out/$tag/ab_wg896.txt"
