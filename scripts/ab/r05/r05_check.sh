#!/usr/bin/env bash
# Round-5 check on one GPU: smoke, the new timed-configuration / instantiation tests, the full GPU suite, the default
# bench line, and a two-rank gloo rehearsal of the multi-rank line (device fields, C5 leg). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05a}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/smoke" 300 python -c "import __graft_entry__ as g; g.smoke()" \
  --- "$tag/newtests" 600 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread \
  --- "$tag/gputest" 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  --- "$tag/bench_c3" 600 python bench.py \
  --- "$tag/rehearse2" 600 python bench.py --gpus 2 --backend gloo --steps 1 --warmup 1 --c5-steps 1 --c5-warmup 0 --no-golden --verify
