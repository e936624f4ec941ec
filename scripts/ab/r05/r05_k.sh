#!/usr/bin/env bash
# Round-5 batch K: the GPU suite (cost-ordered dealing on by default; the mixed kernel's suspendable sphere walk),
# then same-box A/Bs: --cost-order 1 (raster order) against the default on C4 / C3 / C2 with their 8-way emulated
# splits; lib/libhrt_ss0.so (HRT_SPHERE_SUSPEND=0, the sphere walk run to completion) against the product on C5
# (256 spp and the bench line) and C4; suspend_below 16 / 32 on C5; then the diagnostic build's wave records of 1/8
# C4 and C2 shares and the begin-walk lanes on C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05k}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
for cfg in c4 c3 c2; do
  for round in 1 2; do
    for co in 1 0; do
      timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline --no-golden --steps 3 --cost-order $co \
        > "gpurun_out/$tag/${cfg}_co$co.log" 2>&1 || exit 1
      tail -1 "gpurun_out/$tag/${cfg}_co$co.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print('$cfg cost_order $co', d['value'], d['ms_per_step'], e.get('efficiency'), e.get('predicted_ms_per_step'), [r['ms_per_step'] for r in e.get('per_rank', [])])"
    done
  done
done | tee "gpurun_out/$tag/ab_cost_order.txt"
export LIBS="lib/libhrt_ss0.so lib/libhrt.so"
{ bash scripts/ab_lib.sh "--steps 2 --frames 256 --emulate-ranks 0" c5 && bash scripts/ab_lib.sh "--steps 2" c5 \
  && bash scripts/ab_lib.sh "--steps 3 --emulate-ranks 0" c4; } > "gpurun_out/$tag/ab_ss.txt" 2>&1 || exit 1
cat "gpurun_out/$tag/ab_ss.txt"
for sb in 16 32; do
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-golden --steps 2 --frames 256 --emulate-ranks 0 \
    --suspend-below $sb > "gpurun_out/$tag/c5_sb$sb.log" 2>&1 || exit 1
  tail -1 "gpurun_out/$tag/c5_sb$sb.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 256spp suspend_below $sb', d['value'], d['ms_per_step'])"
done
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c4" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 --full \
  --- "$tag/wave_tail_c2" 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 4 0 --full \
  --- "$tag/diag_tris_c5" 300 python scripts/diag_tris.py --frames 16
