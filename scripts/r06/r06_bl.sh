#!/usr/bin/env bash
# Round-6 batch BL: the culling BVH's leaf size re-swept with the two-pass leaf test (lib/libhrt_ml5.so, lib/libhrt_ml6.so:
# -DHRT_BVH_MAX_LEAF=5 / 6) against the default 4. C3, 2 rounds; kernel symbol and tests per ray reported.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06bl}"
mkdir -p "gpurun_out/$tag"
for round in 1 2; do
  for lib in lib/libhrt.so lib/libhrt_ml5.so lib/libhrt_ml6.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
      > "gpurun_out/$tag/c3_$n.log" 2>&1 || exit 1
    echo "c3 $n $(grep '^{"metric' gpurun_out/$tag/c3_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['box_tests_per_ray'], r['sphere_tests_per_ray'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
