#!/usr/bin/env bash
# Round-4 final checks (after the loop-shape changes): the GPU suite, then the default bench line (python bench.py: C3,
# 8-way emulated split) and the C4 / C5 lines with their emulated splits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/final_r04b
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
timeout -k 10 600 python bench.py > $o/bench_c3.log 2>&1 || { tail -20 $o/bench_c3.log; exit 1; }
tail -1 $o/bench_c3.log | cut -c1-300
timeout -k 10 600 python bench.py --config c4 --no-cpu-baseline > $o/bench_c4.log 2>&1 || exit 1
timeout -k 10 900 python bench.py --config c5 --steps 1 --no-cpu-baseline > $o/bench_c5.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline > $o/bench_c1.log 2>&1 && timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > $o/bench_c2.log 2>&1 || exit 1
for c in c1 c2 c3 c4 c5; do tail -1 $o/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'], d['config'].get('launch_frames'), d.get('emulated_split', {}).get('efficiency'))"; done
