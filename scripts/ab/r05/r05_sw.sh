#!/usr/bin/env bash
# Round-5 batch SW: C3 full-image knobs re-checked under the round-5 scheduling (cost order, per-XCD queues): job size
# 32 (default) / 64 and suspend_below 20 / 24 (default) / 28, same box, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag="${1:-r05sw}"
mkdir -p "gpurun_out/$tag"
for round in 1 2; do
  for v in "default:" "jf64:--job-frames 64" "sb20:--suspend-below 20" "sb28:--suspend-below 28"; do
    name="${v%%:*}"; args="${v#*:}"
    timeout -k 10 300 python bench.py --config c3 --steps 3 --emulate-ranks 0 --no-cpu-baseline --no-golden $args > "gpurun_out/$tag/c3_$name.log" 2>&1 || exit 1
    tail -1 "gpurun_out/$tag/c3_$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $name', d['value'], d['ms_per_step'])"
  done
done | tee "gpurun_out/$tag/sweep.txt"
