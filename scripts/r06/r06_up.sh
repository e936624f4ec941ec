#!/usr/bin/env bash
# Round-6 batch UP: the frame block primary rays with their fast sequences guards as wave-uniform branches (product) against
# lib/libhrt_up0.so (HRT_UGUARD_PRIMARY 0). GPU suite first; C3, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06up}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/$tag/gpu_suite.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite.log"; exit 1; }
tail -1 "gpurun_out/$tag/gpu_suite.log"
for round in 1 2 3; do
  for lib in lib/libhrt_up0.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
      > "gpurun_out/$tag/c3_$n.log" 2>&1 || exit 1
    echo "c3 $n $(grep '^{"metric' gpurun_out/$tag/c3_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
