#!/usr/bin/env bash
# Sample buffer vs fold ring at given budgets (bench.py --fold forces the mode).
# usage: scripts/ab_foldmode.sh "<budgets MiB>" <config>...
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/foldmode
budgets="$1"; shift
for cfg in "$@"; do for b in $budgets; do for ring in 0 1; do
  timeout -k 10 300 python bench.py --fold $((ring ? 2 : 1)) --config "$cfg" --no-cpu-baseline --no-golden --steps 2 --warmup 1 \
    --queue-budget-mb "$b" > "gpurun_out/foldmode/${cfg}_${b}_r$ring.log" 2>&1
  echo "$cfg budget=$b ring=$ring $(tail -1 gpurun_out/foldmode/${cfg}_${b}_r$ring.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['fold'], d['config']['fold_bytes'])")"
done; done; done
