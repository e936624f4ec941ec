#!/usr/bin/env bash
# Round-6 batch KP: k_trace's frame-block primary rays (C2) with the fast sequences' guards as wave-uniform branches
# (HRT_UGUARD_KTRACE_PRIMARY, the product build) against lib/libhrt_kp0.so (the guarded functions). GPU suite;
# C2 with its 8-way split, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06kp}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/$tag/gpu_suite.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite.log"; exit 1; }
tail -1 "gpurun_out/$tag/gpu_suite.log"
for round in 1 2 3; do
  for lib in lib/libhrt_kp0.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-golden --steps 10 \
      > "gpurun_out/$tag/c2_$n.log" 2>&1 || exit 1
    echo "c2 $n $(grep '^{"metric' gpurun_out/$tag/c2_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; e=d.get('emulated_split') or {}; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], e.get('efficiency'))")"
  done
done | tee "gpurun_out/$tag/ab_c2.txt"
