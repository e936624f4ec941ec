#!/usr/bin/env bash
# suspend_below x job_frames sweep on one config, one line per run.
# usage: scripts/sweep_suspend.sh <config> "<suspend list>" "<job_frames list>"
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
cfg=$1
for sb in $2; do for jf in $3; do
  timeout -k 10 120 python bench.py --config "$cfg" --steps 2 --warmup 1 --no-cpu-baseline --no-golden \
    --suspend-below "$sb" --job-frames "$jf" > "gpurun_out/sweep/${cfg}_s${sb}_j${jf}.log" 2>&1
  echo "$cfg suspend=$sb jf=$jf $(tail -1 gpurun_out/sweep/${cfg}_s${sb}_j${jf}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
