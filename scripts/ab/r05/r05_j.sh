#!/usr/bin/env bash
# Round-5 batch J: the GPU suite with the suspendable sphere walk of the mixed kernel (k_trace_split_tris<MIXED, BVH, 3>),
# then same-box A/Bs against lib/libhrt_ss0.so (HRT_SPHERE_SUSPEND=0: run to completion in the begin phase) on C5 at
# 256 spp and the full C5 / C4 bench, and the begin-walk lanes of the new form (diagnostic build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05j}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
export LIBS="lib/libhrt_ss0.so lib/libhrt.so"
{ bash scripts/ab_lib.sh "--steps 2 --frames 256 --emulate-ranks 0" c5 && bash scripts/ab_lib.sh "--steps 2" c5 \
  && bash scripts/ab_lib.sh "--steps 3 --emulate-ranks 0" c4; } > "gpurun_out/$tag/ab_ss.txt" 2>&1 || exit 1
cat "gpurun_out/$tag/ab_ss.txt"
for sb in 16 32; do
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-golden --steps 2 --frames 256 --emulate-ranks 0 \
    --suspend-below $sb > "gpurun_out/$tag/c5_sb$sb.log" 2>&1 || exit 1
  tail -1 "gpurun_out/$tag/c5_sb$sb.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 256spp suspend_below $sb', d['value'], d['ms_per_step'])"
done
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/diag_tris_c5" 300 python scripts/diag_tris.py --frames 16
