#!/usr/bin/env bash
# (Historical: measured C5 -1.5 % and not kept; profiles/r04/so/c5leaf_ab.txt.)
# The fast exact sqrt / division in the HL3 mixed kernels' culling-walk leaf test (lib/libhrt.so) against the previous
# commit (lib/libhrt_base.so): the GPU suite, then C5 at full size (two rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/c5leaf_ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # lib cfg tag steps
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps $4 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    > $o/$2_$3.log 2>&1 || return $?
  echo "$3 $2 $(tail -1 $o/$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for round in 1 2; do
  run lib/libhrt_base.so c5 base$round 1 && run lib/libhrt.so c5 new$round 1 || exit 1
done
