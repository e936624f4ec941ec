#!/usr/bin/env bash
# Round-6 batch ML: the mixed kernels' culling sphere walk (C5) with the two-pass leaf and the split kernel's exact fast
# roots (lib/libhrt_ml2.so = -DHRT_MIXED_LEAF2=1) against the one-pass IEEE leaf. GPU tests of the mixed program first;
# C5, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06ml}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_ml2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "gpurun_out/$tag/gpu_suite_ml2.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite_ml2.log"; exit 1; }
tail -1 "gpurun_out/$tag/gpu_suite_ml2.log"
for round in 1 2; do
  for lib in lib/libhrt.so lib/libhrt_ml2.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-golden --steps 1 --warmup 1 --emulate-ranks 0 \
      > "gpurun_out/$tag/c5_$n.log" 2>&1 || exit 1
    echo "c5 $n $(grep '^{"metric' gpurun_out/$tag/c5_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['kernel'])")"
  done
done | tee "gpurun_out/$tag/ab_c5.txt"
