#!/usr/bin/env bash
# Round-5 batch N: the GPU suite with k_trace_steal (frame-block stealing for the linear sphere scan), then same-box
# A/Bs on C2: stealing auto (on for its 1/8 shares) against --steal 1, with the 8-way emulated split, and C3 / C5 checks
# of the final defaults; the diagnostic build's wave records of 1/8 C2 shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05n}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
for round in 1 2; do
  for v in "steal1:--steal 1" "auto:" "steal1_co1:--steal 1 --cost-order 1"; do
    name="${v%%:*}"; args="${v#*:}"
    timeout -k 10 300 python bench.py --config c2 --steps 5 --no-cpu-baseline --no-golden $args > "gpurun_out/$tag/c2_$name.log" 2>&1 || exit 1
    tail -1 "gpurun_out/$tag/c2_$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print('c2 $name', d['value'], d['ms_per_step'], e.get('efficiency'), e.get('predicted_ms_per_step'), [r['ms_per_step'] for r in e.get('per_rank', [])])"
  done
done | tee "gpurun_out/$tag/ab_c2_steal.txt"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c2" 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 4 0 \
  --- "$tag/wave_tail_c2_nosteal" 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 4 0 --steal 1
