#!/usr/bin/env bash
# Round-5 batch RB: row-block size of the row partition (8 = default: whole 8-row tile rows dealt round-robin; 1 = single
# interleaved rows; 2 / 4) on the 8-way emulated splits of C2 / C4 / C3 (the full image is the same in each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag="${1:-r05rb}"
mkdir -p "gpurun_out/$tag"
for round in 1 2; do
  for cfg in c2 c4 c3; do
    for rb in 8 4 2 1; do
      timeout -k 10 300 python bench.py --config $cfg --steps 3 --no-cpu-baseline --no-golden --row-block $rb > "gpurun_out/$tag/${cfg}_rb$rb.log" 2>&1 || exit 1
      tail -1 "gpurun_out/$tag/${cfg}_rb$rb.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print('$cfg rb$rb', d['value'], d['ms_per_step'], e.get('efficiency'), e.get('predicted_ms_per_step'), [r['ms_per_step'] for r in e.get('per_rank', [])])"
    done
  done
done | tee "gpurun_out/$tag/ab_row_block.txt"
