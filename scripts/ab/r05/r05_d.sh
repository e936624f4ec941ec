#!/usr/bin/env bash
# Round-5 batch D: the triangle and tail-split parity tests on the product build (compact 36-B triangle operands,
# tail parts in k_trace's frame-block refill), then same-box A/Bs: C4 / C5 (256 spp) against the 64-B triangle loads
# (lib/libhrt_tri64.so), C2 with its 8-way split. Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05d}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 600 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  "tests/test_gpu_parity.py::test_tail_split_bit_identical" "tests/test_gpu_parity.py::test_hip_reproduces_oracle_fixtures" \
  "tests/test_gpu_parity.py::test_mixed_mode_suzanne_ground_vs_oracle" "tests/test_gpu_parity.py::test_large_mesh_scenes_vs_oracle" \
  "tests/test_gpu_parity.py::test_heap_top_configs_bit_identical" "tests/test_gpu_parity.py::test_tiny_heaps_leaf_pairs_vs_oracle" \
  -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q "failed" "gpurun_out/$tag/tests.log" || exit 1
LIBS="lib/libhrt_tri64.so lib/libhrt.so" bash scripts/ab_lib.sh "--steps 3" c4 > "gpurun_out/$tag/ab_trigeo_c4.txt" 2>&1
cat "gpurun_out/$tag/ab_trigeo_c4.txt"
LIBS="lib/libhrt_tri64.so lib/libhrt.so" bash scripts/ab_lib.sh "--steps 2 --frames 256" c5 > "gpurun_out/$tag/ab_trigeo_c5.txt" 2>&1
cat "gpurun_out/$tag/ab_trigeo_c5.txt"
# WRITE_SIZE calibration of the 12-B sample stores (coalesced vs staggered over 64 rounds), its own PMC pass
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "gpurun_out/$tag/calib" -o calib -- \
  ./hello-raytracing_amd/build/calib_write_size 768 > "gpurun_out/$tag/calib.log" 2>&1 || exit 1
cat "gpurun_out/$tag/calib.log" | grep "{"
find "gpurun_out/$tag/calib" -name "*counter_collection.csv" -exec cat {} \; | cut -c1-400 | head -8
