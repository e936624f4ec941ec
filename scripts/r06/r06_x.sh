#!/usr/bin/env bash
# Round-6 batch X: C5 same-box A/B of the folding waves' placement in the mixed kernel (12-wave workgroups): every
# 64th wave (lib/libhrt.so) against wave 0 of every 5th group of 8 blocks (lib/libhrt_spreadall.so), 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06x}"
mkdir -p "gpurun_out/$tag"
for round in 1 2 3; do
  for lib in lib/libhrt_spreadall.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-golden --steps 1 --warmup 1 --emulate-ranks 0 \
      > "gpurun_out/$tag/c5_$n.log" 2>&1 || exit 1
    echo "c5 $n $(grep '^{"metric' gpurun_out/$tag/c5_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done | tee "gpurun_out/$tag/ab_c5.txt"
