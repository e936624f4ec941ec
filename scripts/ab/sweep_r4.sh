#!/usr/bin/env bash
# Round-4 re-tune of the runtime knobs on the current kernels (interleaved, 2 rounds): suspend_below for C3 / C4 / C5
# (C5 at 512 spp).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
for round in 1 2; do
  for cfg in c3 c4 c5; do
    extra=""; [ $cfg = c5 ] && extra="--frames 512"
    case $cfg in c3) vals="16 20 24 28 32";; *) vals="24 32 40";; esac
    for sb in $vals; do
      timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
        --suspend-below $sb $extra > gpurun_out/sweep/${cfg}_sb${sb}_$round.log 2>&1 || exit $?
      echo "$round $cfg sb=$sb $(tail -1 gpurun_out/sweep/${cfg}_sb${sb}_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
    done
  done
done
