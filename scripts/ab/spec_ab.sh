#!/usr/bin/env bash
# (Historical: the speculative walk measured C3 -7 % and was removed; results in profiles/r04/so/spec_ab.txt.)
# Speculative culling walk (bvh_run_spec, parked leaves; lib/libhrt.so) against the same tree built with
# -DHRT_SPEC=0 (lib/libhrt_nospec.so): the GPU suite, then interleaved C3 lines and a counting C3 line of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/spec_ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # lib cfg tag steps [extra]
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps $4 --warmup 1 --emulate-ranks 0 --no-cpu-baseline \
    --no-golden $5 > $o/$2_$3.log 2>&1 || return $?
  echo "$3 $2 $(tail -1 $o/$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c.get('box_tests_per_ray'), c.get('sphere_tests_per_ray'))")"
}
for round in 1 2 3; do
  run lib/libhrt_nospec.so c3 base$round 3 && run lib/libhrt.so c3 spec$round 3 || exit 1
done
for round in 1 2; do
  run lib/libhrt_nospec.so c2 base$round 3 && run lib/libhrt.so c2 spec$round 3 || exit 1
done
