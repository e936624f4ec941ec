#!/usr/bin/env bash
# C3 after the sign-ordered culling test: suspend_below and job_frames re-checked (the walk step got cheaper).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/sweep_c3_so
mkdir -p $o
run() {  # tag args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden "$@" \
    > $o/$tag.log 2>&1 || return $?
  echo "$tag $(tail -1 $o/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for round in 1 2; do
  for sb in 16 20 24 28 32; do run sb${sb}_$round --suspend-below $sb || exit 1; done
  run jf16_$round --job-frames 16 && run jf64_$round --job-frames 64 || exit 1
done
