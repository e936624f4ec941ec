#!/usr/bin/env bash
# Sample-queue colour-buffer budget sweep (frames per chunk) on the bench configs.
# usage: scripts/sweep_budget.sh "<budgets MiB>" <config>...
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/budget
budgets="$1"; shift
for cfg in "$@"; do
  for b in $budgets; do
    timeout -k 10 300 python bench.py --config "$cfg" --steps 3 --warmup 1 --no-cpu-baseline --no-golden \
      --queue-budget-mb "$b" > "gpurun_out/budget/${cfg}_$b.log" 2>&1
    echo "$cfg $b $(tail -1 gpurun_out/budget/${cfg}_$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
