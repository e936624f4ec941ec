#!/usr/bin/env bash
# Round-6 batch UG: range guards as wave-uniform branches in k_trace_split — candidate roots (leaf pass 2 and the large
# list: HRT_CAND_T 2) and the shading's normal division, normalize and square roots (HRT_UGUARD) — the product build,
# against lib/libhrt_ug0.so (HRT_UGUARD 0) and lib/libhrt_base.so (neither: the branches of the guarded functions).
# GPU suite first; C3, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06ug}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/$tag/gpu_suite.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite.log"; exit 1; }
tail -1 "gpurun_out/$tag/gpu_suite.log"
for round in 1 2 3; do
  for lib in lib/libhrt_base.so lib/libhrt_ug0.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
      > "gpurun_out/$tag/c3_$n.log" 2>&1 || exit 1
    echo "c3 $n $(grep '^{"metric' gpurun_out/$tag/c3_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
