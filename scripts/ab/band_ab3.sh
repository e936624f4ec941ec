#!/usr/bin/env bash
# (Historical: the pipelined band launches this measured were removed after these A/Bs (commit 512dacf); the
# results are in profiles/r04/band/. The lines' config no longer carries a 'bands' field.)
# Bands (8 GiB) with frame-block stealing forced on (short band launches of C4 / C5 trail on a few long jobs), against
# one launch and plain bands; C5 at its full 4096 spp.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bandab3
for round in 1 2; do
  for v in "32768:0" "8192:0" "8192:2"; do
    mb=${v%%:*}; st=${v#*:}
    timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
      --queue-budget-mb $mb --steal $st > gpurun_out/bandab3/c4_${mb}_s${st}_$round.log 2>&1 || exit $?
    echo "$round c4 $mb steal=$st $(tail -1 gpurun_out/bandab3/c4_${mb}_s${st}_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['bands'])")"
  done
done
for v in "32768:0" "8192:0" "8192:2"; do
  mb=${v%%:*}; st=${v#*:}
  timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    --queue-budget-mb $mb --steal $st > gpurun_out/bandab3/c5_${mb}_s${st}.log 2>&1 || exit $?
  echo "c5 $mb steal=$st $(tail -1 gpurun_out/bandab3/c5_${mb}_s${st}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['bands'])")"
done
