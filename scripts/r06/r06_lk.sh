#!/usr/bin/env bash
# Round-6 batch LK: the two-pass leaf with the first candidate's b and disc kept from the first pass (HRT_LEAF_KEEP, the
# product build) against lib/libhrt_lk0.so (every candidate re-read and re-tested). GPU suite; C3, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06lk}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/$tag/gpu_suite.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite.log"; exit 1; }
tail -1 "gpurun_out/$tag/gpu_suite.log"
for round in 1 2 3; do
  for lib in lib/libhrt_lk0.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
      > "gpurun_out/$tag/c3_$n.log" 2>&1 || exit 1
    echo "c3 $n $(grep '^{"metric' gpurun_out/$tag/c3_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; e=d.get('emulated_split') or {}; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], e.get('efficiency'))")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
