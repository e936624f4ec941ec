#!/usr/bin/env bash
# Round-6 batch MX: the mixed kernels — the sphere hit record's guard as a wave-uniform branch (HRT_UGUARD_TRIS) and the
# culling-BVH mixed kernel's heap_begin by refined reciprocals (HRT_HEAP_FAST_BVH) — product build against
# lib/libhrt_mx0.so (neither) and lib/libhrt_mx1.so (the record only). GPU suite; C4 3 rounds, C5 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06mx}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/$tag/gpu_suite.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite.log"; exit 1; }
tail -1 "gpurun_out/$tag/gpu_suite.log"
for round in 1 2 3; do
  for lib in lib/libhrt_mx0.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --no-golden --steps 3 --emulate-ranks 0 \
      > "gpurun_out/$tag/c4_$n.log" 2>&1 || exit 1
    echo "c4 $n $(grep '^{"metric' gpurun_out/$tag/c4_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
  done
done | tee "gpurun_out/$tag/ab_c4.txt"
for round in 1 2; do
  for lib in lib/libhrt_mx0.so lib/libhrt_mx1.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-golden --steps 1 --warmup 1 --emulate-ranks 0 \
      > "gpurun_out/$tag/c5_$n.log" 2>&1 || exit 1
    echo "c5 $n $(grep '^{"metric' gpurun_out/$tag/c5_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
  done
done | tee "gpurun_out/$tag/ab_c5.txt"
