#!/usr/bin/env bash
# Round-6 batch W: the final fold-wave placement — the fold-3 tests and timed compositions, then C3 / C5 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06w}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fold_next.py \
  tests/test_gpu_timed.py > "gpurun_out/$tag/tests.log" 2>&1 || { tail -40 "gpurun_out/$tag/tests.log"; exit 1; }
tail -2 "gpurun_out/$tag/tests.log"
for round in 1 2; do
  timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
    > "gpurun_out/$tag/c3.log" 2>&1 || exit 1
  echo "c3 $(grep '^{"metric' gpurun_out/$tag/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done | tee "gpurun_out/$tag/c3.txt"
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-golden --steps 1 --warmup 1 --emulate-ranks 0 \
  > "gpurun_out/$tag/c5.log" 2>&1 || exit 1
echo "c5 $(grep '^{"metric' gpurun_out/$tag/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee "gpurun_out/$tag/c5.txt"
