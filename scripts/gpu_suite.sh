#!/usr/bin/env bash
# GPU parity suite + a short default bench line, each step under its own time limit (scripts/gpu_step.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag="${1:-suite}"
bash scripts/gpu_step.sh "${tag}_gputest" 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  --- "${tag}_bench_c3" 300 python bench.py --config c3 --steps 3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
  --- "${tag}_bench_c4" 300 python bench.py --config c4 --steps 3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden
