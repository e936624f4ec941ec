#!/usr/bin/env bash
# Grid of suspend_below x job_frames on one config. usage: scripts/exp_grid.sh <config> "<sb list>" "<jf list>" ["<extra>"]
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/grid
cfg="$1"; sbs="$2"; jfs="$3"; extra="${4:-}"
for jf in $jfs; do
  for sb in $sbs; do
    timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline --no-golden --steps 2 --warmup 1 \
      --suspend-below "$sb" --job-frames "$jf" $extra > "gpurun_out/grid/${cfg}_${sb}_$jf.log" 2>&1
    echo "$cfg sb=$sb jf=$jf $(tail -1 gpurun_out/grid/${cfg}_${sb}_$jf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
