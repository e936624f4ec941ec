#!/usr/bin/env bash
# C4 job_frames around its default (32 with the suspendable walks) after the round-4 kernel changes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/sweep_c4_r4
mkdir -p $o
run() {  # tag extra
  timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    $2 > $o/c4_$1.log 2>&1 || return $?
  echo "$1 $(tail -1 $o/c4_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for r in 1 2; do
  run default$r "" && run jf16_$r "--job-frames 16" && run jf64_$r "--job-frames 64" && run jf8_$r "--job-frames 8" || exit 1
done
