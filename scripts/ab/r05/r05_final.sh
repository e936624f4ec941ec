#!/usr/bin/env bash
# Round-5 closing check: the whole GPU suite, smoke(), the default bench line (the driver's command) and the C4 / C2
# bench lines with their 8-way emulated splits, on the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag="${1:-r05_closing}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests_gpu" 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests_gpu.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests_gpu.log" || exit 1
bash scripts/gpu_step.sh "$tag/smoke" 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  --- "$tag/bench" 600 python bench.py \
  --- "$tag/bench_c4" 300 python bench.py --config c4 --steps 3 --no-cpu-baseline --no-golden \
  --- "$tag/bench_c2" 300 python bench.py --config c2 --steps 5 --no-cpu-baseline --no-golden || exit 1
for f in bench bench_c4 bench_c2; do tail -1 "gpurun_out/$tag/$f.log" | cut -c1-400; done
