#!/usr/bin/env bash
# Round-5 batch X: the GPU parity suite on the final tree, a two-rank gloo rehearsal of the multi-rank line on one GPU
# (C3 + the C5 leg, gathered image verified bit for bit; both ranks learn their costs in the warmup), and the default
# bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05x}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
bash scripts/gpu_step.sh "$tag/rehearse2" 600 python bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 --c5-steps 1 \
  --c5-warmup 1 --no-golden --verify \
  --- "$tag/bench" 600 python bench.py
tail -1 "gpurun_out/$tag/rehearse2.log" | cut -c1-600
tail -1 "gpurun_out/$tag/bench.log" | cut -c1-300
