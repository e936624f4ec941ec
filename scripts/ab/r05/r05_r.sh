#!/usr/bin/env bash
# Round-5 batch R (per-XCD job queues): job sizes for short launches — C2 with 4 / 8 / 16-frame jobs, C3 and C4 with
# 16 / 32-frame jobs, each with its 8-way emulated split (the knob applies to the full image and every share).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05r}"
mkdir -p "gpurun_out/$tag"
for round in 1 2; do
  for v in "c2:4" "c2:8" "c2:16" "c3:16" "c3:32" "c4:16" "c4:32"; do
    cfg="${v%%:*}"; jf="${v#*:}"
    timeout -k 10 300 python bench.py --config $cfg --steps 3 --no-cpu-baseline --no-golden --job-frames $jf > "gpurun_out/$tag/${cfg}_jf$jf.log" 2>&1 || exit 1
    tail -1 "gpurun_out/$tag/${cfg}_jf$jf.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print('$cfg jf$jf', d['value'], d['ms_per_step'], e.get('efficiency'), e.get('predicted_ms_per_step'), [r['ms_per_step'] for r in e.get('per_rank', [])])"
  done
done | tee "gpurun_out/$tag/jf_sweep.txt"
