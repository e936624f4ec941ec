#!/usr/bin/env bash
# Round-6 batch Z: C4 (one 512-frame launch + k_accumulate by default) split into 2 or 3 launches that fold each other
# (fold 3 with a 6400 / 4300 MiB budget), 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06z}"
mkdir -p "gpurun_out/$tag"
for round in 1 2; do
  for v in "default:" "two:--fold 3 --queue-budget-mb 6400" "three:--fold 3 --queue-budget-mb 4300"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 $a \
      > "gpurun_out/$tag/c4_$n.log" 2>&1 || exit 1
    echo "c4 $n $(grep '^{"metric' gpurun_out/$tag/c4_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['launch_frames'], c['fold'])")"
  done
done | tee "gpurun_out/$tag/ab_c4.txt"
