#!/usr/bin/env bash
# Round-5 batch I: the GPU suite with cost-ordered dealing on by default (tests/test_gpu_parity.py::
# test_cost_order_bit_identical and every multi-draw test), then same-box A/Bs of --cost-order 1 (raster order, round 4)
# against the default on C4 / C3 / C2 / C5 with their 8-way emulated splits, and the wave records of a 1/8 C4 share
# with cost order (diagnostic build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05i}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
for cfg in c4 c3 c2 c5; do
  steps=3; [ $cfg = c5 ] && steps=2
  for round in 1 2; do
    for co in 1 0; do
      timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline --no-golden --steps $steps --cost-order $co \
        > "gpurun_out/$tag/${cfg}_co$co.log" 2>&1 || exit 1
      tail -1 "gpurun_out/$tag/${cfg}_co$co.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print('$cfg cost_order $co', d['value'], d['ms_per_step'], e.get('efficiency'), e.get('predicted_ms_per_step'), [r['ms_per_step'] for r in e.get('per_rank', [])])"
    done
  done
done | tee "gpurun_out/$tag/ab_cost_order.txt"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c4" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 --full \
  --- "$tag/wave_tail_c2" 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 4 0 --full \
  --- "$tag/diag_tris_c5" 300 python scripts/diag_tris.py --frames 16
