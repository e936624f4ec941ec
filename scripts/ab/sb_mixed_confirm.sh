#!/usr/bin/env bash
# The mixed program's default suspend_below 24: the GPU suite, then the C4 / C5 default lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/sb_mixed_confirm
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --no-golden --emulate-ranks 0 > $o/c4.log 2>&1 &&
timeout -k 10 300 python bench.py --config c5 --steps 1 --no-cpu-baseline --no-golden --emulate-ranks 0 > $o/c5.log 2>&1 || exit 1
for c in c4 c5; do tail -1 $o/$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'], d['roofline'].get('suspend_below'))"; done
