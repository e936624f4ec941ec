#!/usr/bin/env bash
# Round-6 batch SB: suspend_below re-swept on the final kernel (20 / 24 / 28), C3, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06sb}"
mkdir -p "gpurun_out/$tag"
for round in 1 2; do
  for sb in 20 24 28; do
    timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 --suspend-below $sb \
      > "gpurun_out/$tag/c3_sb$sb.log" 2>&1 || exit 1
    echo "c3 sb$sb $(grep '^{"metric' gpurun_out/$tag/c3_sb$sb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
