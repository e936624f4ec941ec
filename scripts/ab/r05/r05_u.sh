#!/usr/bin/env bash
# Round-5 batch U (and Z): the GPU suite with the short-launch policy (half-size jobs, cost order instead of stealing for a
# row partition's shares), then the default bench lines of C4 / C3 / C2 / C5 with their 8-way emulated splits, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05u}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
for round in 1 2; do
  for cfg in c4 c3 c2 c5; do
    steps=3; [ $cfg = c5 ] && steps=2
    timeout -k 10 400 python bench.py --config $cfg --steps $steps --no-cpu-baseline --no-golden > "gpurun_out/$tag/${cfg}.log" 2>&1 || exit 1
    tail -1 "gpurun_out/$tag/${cfg}.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print('$cfg', d['value'], d['ms_per_step'], e.get('efficiency'), e.get('predicted_ms_per_step'), [r['ms_per_step'] for r in e.get('per_rank', [])])"
  done
done | tee "gpurun_out/$tag/defaults.txt"
