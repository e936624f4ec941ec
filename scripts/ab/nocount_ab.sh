#!/usr/bin/env bash
# Cost of the per-lane work counters (box / sphere tests) in the culling walks: the same tree with the counting
# compiled out (lib/libhrt_nc.so; its bench lines report no rays: compare ms_per_step) against lib/libhrt.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/nocount_ab
mkdir -p $o
run() {  # lib cfg tag steps [args]
  local lib=$1 cfg=$2 tag=$3 steps=$4; shift 4
  HRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden "$@" \
    > $o/${cfg}_$tag.log 2>&1 || return $?
  echo "$cfg $tag $lib $(grep -o '"ms_per_step": [0-9.]*' $o/${cfg}_$tag.log)"
}
for round in 1 2 3; do
  run lib/libhrt.so c3 count$round 3 && run lib/libhrt_nc.so c3 nocount$round 3 || exit 1
done
run lib/libhrt.so c5 count 1 --frames 256 && run lib/libhrt_nc.so c5 nocount 1 --frames 256
