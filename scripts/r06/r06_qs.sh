#!/usr/bin/env bash
# Round-6 batch QS: the launch-end tail and the drain's queue scan. A wave whose XCD's job queue runs dry tries the other
# seven queues with one atomic each before it exits; at the drain that is ~8 failing atomics per wave on 8 addresses.
# lib/libhrt_q1.so (-DHRT_QSCAN=1): own queue only (every XCD's waves drain their own queue); lib/libhrt_q2.so: own + the
# next. C2 and C3 with their 8-way emulated splits, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06qs}"
mkdir -p "gpurun_out/$tag"
for cfg in c2 c3; do
  for round in 1 2; do
    for lib in lib/libhrt.so lib/libhrt_q1.so lib/libhrt_q2.so; do
      n=$(basename $lib .so)
      HRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-golden --steps 5 \
        > "gpurun_out/$tag/${cfg}_$n.log" 2>&1 || exit 1
      echo "$cfg $n $(grep '^{"metric' gpurun_out/$tag/${cfg}_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; e=d.get('emulated_split') or {}; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], e.get('efficiency'), e.get('predicted_ms_per_step'), e.get('bitwise_equal_full_image'))")"
    done
  done
done | tee "gpurun_out/$tag/ab.txt"
