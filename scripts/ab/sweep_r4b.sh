#!/usr/bin/env bash
# After the loop-shape changes: the signed-pad near / far constants (lib/libhrt.so) against the previous commit
# (lib/libhrt_base.so) on C3 and C5, then C3's suspend_below and job_frames re-checked around the defaults (24, 32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/sweep_r4b
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # lib cfg tag steps [extra]
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps $4 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    $5 > $o/$2_$3.log 2>&1 || return $?
  echo "$3 $2 $(tail -1 $o/$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for round in 1 2; do
  run lib/libhrt_base.so c3 base$round 3 && run lib/libhrt.so c3 new$round 3 || exit 1
done
run lib/libhrt_base.so c5 base1 1 && run lib/libhrt.so c5 new1 1 || exit 1
for sb in 16 20 28 32; do run lib/libhrt.so c3 sb$sb 3 "--suspend-below $sb" || exit 1; done
for jf in 16 64; do run lib/libhrt.so c3 jf$jf 3 "--job-frames $jf" || exit 1; done
run lib/libhrt.so c3 default 3
