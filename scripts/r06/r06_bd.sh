#!/usr/bin/env bash
# Round-6 batch BD: two branch removals in k_trace_split — bvh_begin's coverage test as a select (HRT_BEGIN_SELECT) and the
# descent as one while loop instead of a do-while inside an if (HRT_DESCENT_WHILE) — the product build (both) against
# lib/libhrt_b00.so (neither), lib/libhrt_b10.so (select only), lib/libhrt_b01.so (while only). GPU suite; C3, 3 rounds;
# C5 (the mixed kernels' sphere walk shares the descent), 2 rounds of the product and b00.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06bd}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/$tag/gpu_suite.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite.log"; exit 1; }
tail -1 "gpurun_out/$tag/gpu_suite.log"
for round in 1 2 3; do
  for lib in lib/libhrt_b00.so lib/libhrt_b10.so lib/libhrt_b01.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
      > "gpurun_out/$tag/c3_$n.log" 2>&1 || exit 1
    echo "c3 $n $(grep '^{"metric' gpurun_out/$tag/c3_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
for round in 1 2; do
  for lib in lib/libhrt_b00.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-golden --steps 1 --warmup 1 --emulate-ranks 0 \
      > "gpurun_out/$tag/c5_$n.log" 2>&1 || exit 1
    echo "c5 $n $(grep '^{"metric' gpurun_out/$tag/c5_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
  done
done | tee "gpurun_out/$tag/ab_c5.txt"
