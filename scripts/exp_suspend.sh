#!/usr/bin/env bash
# A/B of k_trace_split's suspend threshold on a bench config (sample queue, culling BVH).
# usage: scripts/exp_suspend.sh <config> <thresholds...>
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/suspend
cfg="$1"; shift
for sb in "$@"; do
  timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline --steps 2 --warmup 1 --suspend-below "$sb" \
    > "gpurun_out/suspend/${cfg}_$sb.log" 2>&1
  echo "$cfg suspend_below=$sb $(tail -1 gpurun_out/suspend/${cfg}_$sb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
done
