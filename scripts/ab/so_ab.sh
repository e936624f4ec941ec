#!/usr/bin/env bash
# Sign-ordered heap-top layout (lib/libhrt.so) against the previous tree (lib/libhrt_base.so): the GPU suite on the
# new build, then interleaved C4 / C5 (256 spp) bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/so_ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -2 $o/gputest.log
run() {  # lib cfg tag steps [extra]
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps $4 --warmup 1 --emulate-ranks 0 --no-cpu-baseline \
    --no-golden $5 > $o/$2_$3.log 2>&1 || return $?
  echo "$3 $2 $1 $(tail -1 $o/$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'])")"
}
for round in 1 2; do
  run lib/libhrt_base.so c4 base$round 3 && run lib/libhrt.so c4 so$round 3 || exit 1
  run lib/libhrt_base.so c5 base$round 1 "--frames 256" && run lib/libhrt.so c5 so$round 1 "--frames 256" || exit 1
done
