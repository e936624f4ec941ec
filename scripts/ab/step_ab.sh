#!/usr/bin/env bash
# The heap walk's step count materialised once per trip (no loop-latch copy; lib/libhrt.so) against the previous
# commit (lib/libhrt_base.so): the GPU suite, then interleaved C4 and C5 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/step_ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # lib cfg tag steps
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps $4 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    > $o/$2_$3.log 2>&1 || return $?
  echo "$3 $2 $(tail -1 $o/$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for round in 1 2 3; do
  run lib/libhrt_base.so c4 base$round 3 && run lib/libhrt.so c4 new$round 3 || exit 1
done
run lib/libhrt_base.so c5 base1 1 && run lib/libhrt.so c5 new1 1
