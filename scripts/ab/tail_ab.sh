#!/usr/bin/env bash
# Tail split off (1) / quarters (2) / eighths (3), now in the triangle / mixed kernels too: C3, C4, C5 (4096 spp);
# the tail-split parity test first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/tail_ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "tail_split or heap_top or oracle" > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # cfg tag steps args
  local cfg=$1 tag=$2 steps=$3; shift 3
  timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden "$@" \
    > $o/${cfg}_$tag.log 2>&1 || return $?
  echo "$cfg $tag $(tail -1 $o/${cfg}_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for round in 1 2; do
  for t in 1 2 3; do run c4 t${t}_$round 3 --tail-split $t || exit 1; done
  for t in 2 3; do run c3 t${t}_$round 3 --tail-split $t || exit 1; done
done
for t in 1 2 3; do run c5 t$t 1 --tail-split $t || exit 1; done
