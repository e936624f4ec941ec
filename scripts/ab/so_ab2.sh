#!/usr/bin/env bash
# Sign-ordered heap top: 971 nodes (lib/libhrt.so) vs 881 (lib/libhrt_ht881.so) vs the previous tree
# (lib/libhrt_base.so), interleaved C4 / C5 (256 spp) bench lines; parity suite on the default build first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/so_ab2
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tri or mixed or suzan or heap or leaf or oracle" > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # lib cfg tag steps [extra]
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps $4 --warmup 1 --emulate-ranks 0 --no-cpu-baseline \
    --no-golden $5 > $o/$2_$3.log 2>&1 || return $?
  echo "$3 $2 $1 $(tail -1 $o/$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for round in 1 2; do
  for v in base:lib/libhrt_base.so ht971:lib/libhrt.so ht881:lib/libhrt_ht881.so; do
    run ${v#*:} c4 ${v%%:*}$round 3 || exit 1
  done
  for v in base:lib/libhrt_base.so ht971:lib/libhrt.so ht881:lib/libhrt_ht881.so; do
    run ${v#*:} c5 ${v%%:*}$round 1 "--frames 256" || exit 1
  done
done
