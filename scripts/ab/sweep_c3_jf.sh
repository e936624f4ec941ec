#!/usr/bin/env bash
# C3 with launches of whole jobs (352 + 352 + 320 frames: the tail split applies again): job_frames 16 / 32, and the
# chunk test; then the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/sweep_c3_jf
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # tag args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden "$@" \
    > $o/$tag.log 2>&1 || return $?
  echo "$tag $(tail -1 $o/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['launch_frames'])")"
}
for round in 1 2; do
  run jf32_$round && run jf16_$round --job-frames 16 && run jf32_sb20_$round --suspend-below 20 || exit 1
done
