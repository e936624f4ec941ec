#!/usr/bin/env bash
# C5 (full 4K x 4096) around its defaults after the round-4 kernel changes: suspend_below 24 / 32 (default) / 40 / 48,
# job_frames 8 / 32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/sweep_c5_r4
mkdir -p $o
run() {  # tag extra
  timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    $2 > $o/c5_$1.log 2>&1 || return $?
  echo "$1 $(tail -1 $o/c5_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
run default "" && run sb24 "--suspend-below 24" && run sb40 "--suspend-below 40" && run sb48 "--suspend-below 48" &&
run jf8 "--job-frames 8" && run jf32 "--job-frames 32" && run default2 ""
