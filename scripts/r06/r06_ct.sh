#!/usr/bin/env bash
# Round-6 batch CT: the candidate root with its range guards as one wave-uniform branch (candidate_t): in the two-pass
# leaf's second pass (HRT_CAND_T 1, the product build) and also for the large list in bvh_begin (lib/libhrt_ct2.so),
# against exact_t_geo's branches (lib/libhrt_ct0.so). GPU suite on the product and ct2 builds; C3, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06ct}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/$tag/gpu_suite.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite.log"; exit 1; }
tail -1 "gpurun_out/$tag/gpu_suite.log"
HRT_LIB=lib/libhrt_ct2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sphere or golden or culling or c3 or suspend or cost or timed or packet or fold or split" > "gpurun_out/$tag/gpu_suite_ct2.log" 2>&1 || { tail -30 "gpurun_out/$tag/gpu_suite_ct2.log"; exit 1; }
tail -1 "gpurun_out/$tag/gpu_suite_ct2.log"
for round in 1 2 3; do
  for lib in lib/libhrt_ct0.so lib/libhrt.so lib/libhrt_ct2.so; do
    n=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
      > "gpurun_out/$tag/c3_$n.log" 2>&1 || exit 1
    echo "c3 $n $(grep '^{"metric' gpurun_out/$tag/c3_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
