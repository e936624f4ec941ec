#!/usr/bin/env bash
# Round-5 batch O: the GPU suite, then same-box A/Bs of stealing on C2 shares (k_trace_steal; auto against --steal 1,
# with / without the cost order) and on full images (--steal 2 against auto: C2, C3, C4); the diagnostic build's wave
# records of 1/8 C2 shares with and without stealing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05o}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
for round in 1 2; do
  for v in "c2:steal1:--steal 1" "c2:auto:" "c2:steal1_co1:--steal 1 --cost-order 1" "c2:steal2:--steal 2 --emulate-ranks 0" \
           "c3:steal2:--steal 2 --emulate-ranks 0" "c3:auto0:--emulate-ranks 0" "c4:steal2:--steal 2 --emulate-ranks 0" "c4:auto0:--emulate-ranks 0"; do
    cfg="${v%%:*}"; rest="${v#*:}"; name="${rest%%:*}"; args="${rest#*:}"
    timeout -k 10 300 python bench.py --config $cfg --steps 3 --no-cpu-baseline --no-golden $args > "gpurun_out/$tag/${cfg}_$name.log" 2>&1 || exit 1
    tail -1 "gpurun_out/$tag/${cfg}_$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print('$cfg $name', d['value'], d['ms_per_step'], e.get('efficiency'), e.get('predicted_ms_per_step'), [r['ms_per_step'] for r in e.get('per_rank', [])])"
  done
done | tee "gpurun_out/$tag/ab_steal.txt"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c2" 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 4 0 \
  --- "$tag/wave_tail_c2_nosteal" 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 4 0 --steal 1
