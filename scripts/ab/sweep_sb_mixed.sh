#!/usr/bin/env bash
# suspend_below for the mixed program (C4: linear sphere scan + heap walk; C5: culling-BVH sphere walk + heap walk)
# around the default 32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/sweep_sb_mixed
mkdir -p $o
run() {  # cfg tag steps extra
  timeout -k 10 300 python bench.py --config $1 --steps $3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    $4 > $o/$1_$2.log 2>&1 || return $?
  echo "$2 $1 $(tail -1 $o/$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for sb in 32 24 28 20; do run c4 sb$sb 3 "--suspend-below $sb" || exit 1; done
for sb in 16 20 24 28; do run c5 sb$sb 1 "--suspend-below $sb" || exit 1; done
run c4 sb32b 3 "--suspend-below 32" && run c4 sb24b 3 "--suspend-below 24" && run c5 sb32 1 "--suspend-below 32"
