#!/usr/bin/env bash
# Round-5 final check A: the whole GPU suite, smoke(), the default bench line (the driver's command) on the final tree,
# and the diagnostic build's wave records of 1/8 C2 and C4 shares with the final defaults.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05_final}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests_gpu" 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests_gpu.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests_gpu.log" || exit 1
bash scripts/gpu_step.sh "$tag/smoke" 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  --- "$tag/bench" 600 python bench.py || exit 1
tail -1 "gpurun_out/$tag/bench.log"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c2" 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 4 --full \
  --- "$tag/wave_tail_c4" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0
