#!/usr/bin/env bash
# Round-5 batch G: parity tests on the product build (tail claim rule for tail parts), then same-box A/Bs of the rule
# (lib/libhrt_tc0.so = HRT_TAIL_CLAIM=0, round 4) on C3, C4 without stealing and C5, with their 8-way emulated splits
# (ab_lib.sh prints: value, ms/step, emulated efficiency, predicted ms/step); then C4's 8-way split under the
# short-launch options (the bench knobs apply to the full image and every share) and the wave records of a 1/8 C4 share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05g}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
export LIBS="lib/libhrt_tc0.so lib/libhrt.so"
{ bash scripts/ab_lib.sh "--steps 3" c3 && bash scripts/ab_lib.sh "--steps 3 --steal 1" c4 \
  && bash scripts/ab_lib.sh "--steps 2" c5; } > "gpurun_out/$tag/ab_tc.txt" 2>&1 || exit 1
cat "gpurun_out/$tag/ab_tc.txt"
for v in "auto:" "nosteal8:--steal 1 --tail-split 3" "jf16:--job-frames 16" "jf16nosteal:--job-frames 16 --steal 1"; do
  name="${v%%:*}"; args="${v#*:}"
  bash scripts/gpu_step.sh "$tag/c4_$name" 300 python bench.py --config c4 --no-cpu-baseline --no-golden --steps 3 $args \
    > /dev/null || exit 1
  tail -1 "gpurun_out/$tag/c4_$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['emulated_split']; print('c4 $name', d['value'], d['ms_per_step'], e['efficiency'], e['predicted_ms_per_step'], [r['ms_per_step'] for r in e['per_rank']])"
done
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c4" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 \
  --- "$tag/wave_tail_c4_nosteal" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 --steal 1
