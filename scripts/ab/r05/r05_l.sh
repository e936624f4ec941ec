#!/usr/bin/env bash
# Round-5 batch L: the GPU suite with cost-ordered dealing as a stable head / rest partition (the most expensive
# quarter of the tiles first, each part in raster order), then same-box A/Bs of --cost-order 1 (raster order) against
# the default on C4 / C3 / C2 with their 8-way emulated splits and on C5 (256 spp, and the bench line), and the
# diagnostic build's wave records of 1/8 C4 and C2 shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05l}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
for cfg in c4 c3 c2 c5s c5; do
  case $cfg in c5s) args="--config c5 --steps 2 --frames 256 --emulate-ranks 0";; c5) args="--config c5 --steps 2";;
    *) args="--config $cfg --steps 3";; esac
  for round in 1 2; do
    for co in 1 0; do
      timeout -k 10 400 python bench.py $args --no-cpu-baseline --no-golden --cost-order $co \
        > "gpurun_out/$tag/${cfg}_co$co.log" 2>&1 || exit 1
      tail -1 "gpurun_out/$tag/${cfg}_co$co.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print('$cfg cost_order $co', d['value'], d['ms_per_step'], e.get('efficiency'), e.get('predicted_ms_per_step'), [r['ms_per_step'] for r in e.get('per_rank', [])])"
    done
  done
done | tee "gpurun_out/$tag/ab_cost_order.txt"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c4" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 --full \
  --- "$tag/wave_tail_c2" 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 4 0 --full
