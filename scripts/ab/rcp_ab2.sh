#!/usr/bin/env bash
# C5 at full size and C4: previous commit (libhrt_base.so) vs refined 1/det only (libhrt_tri.so) vs 1/det and the heap
# walk's 1/d (libhrt.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/rcp_ab2
mkdir -p $o
run() {  # lib cfg tag steps [extra]
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps $4 --warmup 1 --emulate-ranks 0 --no-cpu-baseline \
    --no-golden $5 > $o/$2_$3.log 2>&1 || return $?
  echo "$3 $2 $(tail -1 $o/$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for round in 1 2; do
  run lib/libhrt_base.so c5 base$round 1 && run lib/libhrt_tri.so c5 tri$round 1 && run lib/libhrt.so c5 both$round 1 || exit 1
done
for round in 1 2; do
  run lib/libhrt_base.so c4 base$round 3 && run lib/libhrt_tri.so c4 tri$round 3 && run lib/libhrt.so c4 both$round 3 || exit 1
done
