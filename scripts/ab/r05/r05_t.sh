#!/usr/bin/env bash
# Round-5 batch T: the GPU suite with the cost order's head sorted by cost class, then C4 8-way splits under stealing
# (the default) against cost order without stealing (32- and 16-frame jobs), C3 and C2 (8-frame jobs) for reference,
# and the wave records of C4's 1/8 shares 4 / 0 / 5 without stealing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05t}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
for round in 1 2; do
  for v in "c4:steal:" "c4:co_jf32:--steal 1" "c4:co_jf16:--steal 1 --job-frames 16" "c3:default:" "c2:jf8:--job-frames 8"; do
    cfg="${v%%:*}"; rest="${v#*:}"; name="${rest%%:*}"; args="${rest#*:}"
    timeout -k 10 300 python bench.py --config $cfg --steps 3 --no-cpu-baseline --no-golden $args > "gpurun_out/$tag/${cfg}_$name.log" 2>&1 || exit 1
    tail -1 "gpurun_out/$tag/${cfg}_$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print('$cfg $name', d['value'], d['ms_per_step'], e.get('efficiency'), e.get('predicted_ms_per_step'), [r['ms_per_step'] for r in e.get('per_rank', [])])"
  done
done | tee "gpurun_out/$tag/ab_order.txt"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/c4_jf16" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 5 --param job_frames=16 --param steal=1
