#!/usr/bin/env bash
# Round-6 batch LU: the two-pass leaf's first pass unrolled (HRT_LEAF_UNROLL 2 / 4: lib/libhrt_u2.so, lib/libhrt_u4.so)
# and suspend_below re-swept with the two-pass leaf (20 / 24 / 28 / 32). C3, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06lu}"
mkdir -p "gpurun_out/$tag"
run() {  # name lib extra-args
  HRT_LIB=$2 timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 $3 \
    > "gpurun_out/$tag/c3_$1.log" 2>&1 || exit 1
  echo "c3 $1 $(grep '^{"metric' gpurun_out/$tag/c3_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
}
for round in 1 2; do
  run base lib/libhrt.so ""
  run u2 lib/libhrt_u2.so ""
  run u4 lib/libhrt_u4.so ""
  for sb in 20 28 32; do run sb$sb lib/libhrt.so "--suspend-below $sb"; done
done | tee "gpurun_out/$tag/ab_c3.txt"
