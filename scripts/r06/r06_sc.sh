#!/usr/bin/env bash
# Round-6 batch SC: k_trace's simple sphere scan in two passes (HRT_SCAN_2PASS: discriminant tests of every slot, then
# the exact roots of each lane's candidates; HRT_SCAN_FAST: those roots by the range-guarded exact sequences) against
# the one-pass scan (lib/libhrt_noscan.so) and the two-pass scan with IEEE roots (lib/libhrt_scanieee.so). C2 with its
# 8-way emulated split, 2 rounds; the sphere-program GPU tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06sc}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/$tag/gpu_suite.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite.log"; exit 1; }
tail -3 "gpurun_out/$tag/gpu_suite.log"
for round in 1 2; do
  for lib in lib/libhrt_noscan.so lib/libhrt_scanieee.so lib/libhrt.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-golden --steps 10 \
      > "gpurun_out/$tag/c2_$n.log" 2>&1 || exit 1
    echo "c2 $n $(grep '^{"metric' gpurun_out/$tag/c2_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; e=d.get('emulated_split') or {}; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['kernel'], e.get('efficiency'))")"
  done
done | tee "gpurun_out/$tag/ab_c2.txt"
HRT_LIB=lib/libhrt.so timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
  > "gpurun_out/$tag/c3.log" 2>&1 || exit 1
grep '^{"metric' gpurun_out/$tag/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['ms_per_step'])"
