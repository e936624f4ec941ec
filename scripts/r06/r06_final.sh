#!/usr/bin/env bash
# Round-6 closing check on one GPU: smoke, the full GPU suite, the default bench line, the other configs' lines and a
# two-rank gloo rehearsal of the multi-rank line (device fields, gather checksum, C5 leg). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06fin}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/smoke" 300 python -c "import __graft_entry__ as g; g.smoke()" \
  --- "$tag/gputest" 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  --- "$tag/bench_c3" 600 python bench.py \
  --- "$tag/bench_c2" 300 python bench.py --config c2 --steps 10 --no-cpu-baseline --no-golden \
  --- "$tag/bench_c4" 300 python bench.py --config c4 --steps 3 --no-cpu-baseline --no-golden \
  --- "$tag/bench_c5" 600 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-golden \
  --- "$tag/rehearse2" 600 python bench.py --gpus 2 --backend gloo --steps 1 --warmup 1 --c5-steps 1 --c5-warmup 0 --no-golden --verify
