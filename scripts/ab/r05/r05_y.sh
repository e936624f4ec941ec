#!/usr/bin/env bash
# Round-5 batch Y: full images in cost order (--cost-order 2: the costly half of the tiles first, sorted; learnt in the
# warmup) against raster order (--cost-order 1, the full-image default), C3 / C4 / C2 / C5 (256 spp), same box, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05y}"
mkdir -p "gpurun_out/$tag"
for round in 1 2; do
  for cfg in c3 c4 c2 c5s; do
    case $cfg in c5s) args="--config c5 --steps 2 --frames 256";; c2) args="--config c2 --steps 5";; *) args="--config $cfg --steps 3";; esac
    for co in 1 2; do
      timeout -k 10 300 python bench.py $args --emulate-ranks 0 --no-cpu-baseline --no-golden --cost-order $co \
        > "gpurun_out/$tag/${cfg}_co$co.log" 2>&1 || exit 1
      tail -1 "gpurun_out/$tag/${cfg}_co$co.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg cost_order $co', d['value'], d['ms_per_step'])"
    done
  done
done | tee "gpurun_out/$tag/ab_full_order.txt"
