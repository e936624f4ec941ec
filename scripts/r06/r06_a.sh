#!/usr/bin/env bash
# Round-6 batch A: the packet walk of primary rays (k_trace_split<.., PACKET>) — GPU suite on the product build, then
# a same-box A/B on C3: packet off / on (product library, rt_params.packet 1 / 2) and every k_trace_split at 6 waves
# with the packet off (lib/libhrt_w6.so: the cost of the packet kernel's 6 waves alone). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06a}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/timed" 400 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread \
  --- "$tag/gputest" 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
for round in 1 2; do
  for v in "lib/libhrt.so 1" "lib/libhrt.so 2" "lib/libhrt_w6.so 1"; do
    set -- $v
    HRT_LIB="$1" timeout -k 10 300 python bench.py --config c3 --steps 5 --no-cpu-baseline --no-golden --packet "$2" \
      > "gpurun_out/$tag/c3_$(basename $1 .so)_p$2_$round.log" 2>&1 || exit 1
    echo "c3 $1 packet $2 round $round: $(tail -1 gpurun_out/$tag/c3_$(basename $1 .so)_p$2_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done | tee "gpurun_out/$tag/ab.txt"
