#!/usr/bin/env bash
# Round-5 batch F: parity tests on the product build (tail claim rule, compact triangle operands, k_trace tail parts),
# then same-box A/Bs: C4's 8-way emulated split by tail claim rule (CLAIM_FREE 0 = round 4 / 32 = product / 48; STEAL_OWN 1),
# the compact triangle operands on C4 / C5 (256 spp), C2 with / without tail parts; then the WRITE_SIZE calibration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05f}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/tests" 900 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/tests.log" && ! grep -q -E "[0-9]+ failed" "gpurun_out/$tag/tests.log" || exit 1
LIBS="lib/libhrt_cf0.so lib/libhrt.so lib/libhrt_cf48.so lib/libhrt_cf32o1.so" bash scripts/ab_lib.sh "--steps 3" c4 \
  > "gpurun_out/$tag/ab_claim_c4.txt" 2>&1
for f in gpurun_out/ab/c4_libhrt*.log; do tail -1 "$f" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['emulated_split']; print('$f', d['value'], e['efficiency'], e['predicted_ms_per_step'])"; done >> "gpurun_out/$tag/ab_claim_c4.txt"
cat "gpurun_out/$tag/ab_claim_c4.txt"
LIBS="lib/libhrt_tri64.so lib/libhrt.so" bash scripts/ab_lib.sh "--steps 2 --frames 256 --emulate-ranks 0" c5 > "gpurun_out/$tag/ab_trigeo_c5.txt" 2>&1
cat "gpurun_out/$tag/ab_trigeo_c5.txt"
LIBS="lib/libhrt_tri64.so lib/libhrt.so" bash scripts/ab_lib.sh "--steps 3 --emulate-ranks 0" c4 > "gpurun_out/$tag/ab_trigeo_c4.txt" 2>&1
cat "gpurun_out/$tag/ab_trigeo_c4.txt"
for r in 1 2; do for t in 1 0; do
  timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-golden --steps 5 --tail-split $t > "gpurun_out/$tag/c2_tail$t.log" 2>&1 || exit 1
  tail -1 "gpurun_out/$tag/c2_tail$t.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['emulated_split']; print('c2 tail_split $t', d['value'], d['ms_per_step'], e['efficiency'], e['predicted_ms_per_step'])"
done; done
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "gpurun_out/$tag/calib" -o calib -- \
  ./hello-raytracing_amd/build/calib_write_size 768 > "gpurun_out/$tag/calib.log" 2>&1 || exit 1
grep "{" "gpurun_out/$tag/calib.log"
find "gpurun_out/$tag/calib" -name "*counter_collection.csv" -exec cat {} \; | cut -c1-400 | head -8
