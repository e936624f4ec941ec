#!/usr/bin/env bash
# k_trace_split's culling walk with the descent as a bottom-tested loop (lib/libhrt.so) against the same tree built
# with -DHRT_BTEST=0 (lib/libhrt_nobt.so, the top-tested loop): the GPU suite, then interleaved C3 and C2 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/btest_ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # lib cfg tag
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps 3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    > $o/$2_$3.log 2>&1 || return $?
  echo "$3 $2 $(tail -1 $o/$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c.get('box_tests_per_ray'), c.get('sphere_tests_per_ray'))")"
}
for round in 1 2 3; do
  run lib/libhrt_nobt.so c3 base$round && run lib/libhrt.so c3 bt$round || exit 1
done
for round in 1 2; do
  run lib/libhrt_nobt.so c2 base$round && run lib/libhrt.so c2 bt$round || exit 1
done
